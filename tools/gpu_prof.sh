# Tests, bench (twice), then a rocprofv3 kernel trace of a short bench run summarised
# per kernel and per (kernel, grid).  usage: bash tools/gpu_prof.sh <outdir> "<pytest targets>"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread $2 > $O/t.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/t.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 0; fi
fi
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$rep.json 2> $O/bench_$rep.err || { echo "bench failed"; exit 0; }
  python -c "import json; d=json.load(open('$O/bench_$rep.json')); print('bench', d['value'], {k.split(':')[0]: v['mean_ms'] for k, v in d['roofline']['per_kernel'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --kernel-steps 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 0; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py $T --steps 8 > $O/summary.md && python tools/prof_summary.py $T --steps 8 --by-grid > $O/summary_by_grid.md
head -30 $O/summary.md
echo ALLDONE
