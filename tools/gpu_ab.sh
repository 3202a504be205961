# Time conv microbench cases against several library builds (A/B experiments).
# usage: bash tools/gpu_ab.sh <outdir> "<bench_conv args>" lib1 lib2 ...   ("base" = libirgan.so)
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; ARGS=$2; shift 2
mkdir -p $O
P=infrared-colorization-with-resnet-generator-and-patchgan_amd
for L in "$@"; do
  if [ "$L" = base ]; then LIB=$P/libirgan.so; else LIB=$P/build/libirgan_$L.so; fi
  echo "## $L" >> $O/ab.txt
  IRGAN_LIB=$LIB timeout -k 10 120 python tools/bench_conv.py $ARGS >> $O/ab.txt 2>&1
done
cat $O/ab.txt
echo ALLDONE
