# Full GPU tests, then bench.py A/B across env settings (each run twice, interleaved).
# usage: bash tools/gpu_ab_bench.sh <outdir> "ENV=a" "-" ...   ("-" = no extra env)
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
for rep in 1 2; do
  for E in "$@"; do
    T=$(echo "$E" | tr '= ' '__')
    if [ "$E" = "-" ]; then E=""; fi
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_${T}_$rep.json 2> $O/bench_${T}_$rep.err
    echo "$E rep$rep $(python -c "import json,sys; d=json.load(open('$O/bench_${T}_$rep.json')); print(d['value'], d['ms_per_step_median'])")" >> $O/ab.txt
  done
done
cat $O/ab.txt
echo ALLDONE
