# Full GPU check (tests, smoke, bench, rocprof) plus one A/B bench line with an env
# switch.  usage: bash tools/gpu_full_ab.sh <outdir-name> <ENV=VALUE>
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-full}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
env $2 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_ab.json 2> $O/bench_ab.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
echo ALLDONE
