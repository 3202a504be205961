# Time conv microbench cases under several environment settings (runtime A/B knobs).
# usage: bash tools/gpu_env_ab.sh <outdir> "<bench_conv args>" "ENV1=a ENV2=b" "ENV3=c" ...  ("-" = no extra env)
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; ARGS=$2; shift 2
mkdir -p $O
for E in "$@"; do
  echo "## $E" >> $O/ab.txt
  if [ "$E" = "-" ]; then E=""; fi
  env $E timeout -k 10 120 python tools/bench_conv.py $ARGS >> $O/ab.txt 2>&1
done
cat $O/ab.txt
echo ALLDONE
