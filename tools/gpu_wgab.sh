# wgrad_pc variant A/B: microbench (resblock + up2 shapes), parity subset, then PMC traffic of
# the default build's wgrad.  usage: bash tools/gpu_wgab.sh <outdir> <variant> ...
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
B=infrared-colorization-with-resnet-generator-and-patchgan_amd/variants
for v in default "$@"; do
  L=""; [ $v != default ] && L=$B/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 120 python tools/bench_conv.py --case res3x3 --which wgrad --iters 50 > $O/mb_$v.txt 2>&1 || { echo "$v failed"; exit 1; }
  echo "$v: $(tail -1 $O/mb_$v.txt)"
done
echo ALLDONE
