# Same-box A/B of environment switches on the default bench: each arm twice, interleaved.
# usage: [BENCH_EXTRA="--batch 32 --dtype fp8"] bash tools/gpu_envab.sh <outdir-name> "<arm env 1>" ... ("-" = no env)
export TMPDIR=/tmp
N=${1:-envab}; shift
O=gpurun_out/$N
mkdir -p $O
for rep in 1 2; do
  i=0
  for arm in "$@"; do
    i=$((i+1))
    if [ "$arm" = "-" ]; then E=""; else E="$arm"; fi
    env $E timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline $BENCH_EXTRA > $O/arm${i}_$rep.json 2> $O/arm${i}_$rep.err || { echo "arm $i failed"; tail -3 $O/arm${i}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/arm${i}_$rep.json')); print('arm $i ($arm) rep $rep', d['value'], d['ms_per_step'])"
  done
done
echo AB_DONE
