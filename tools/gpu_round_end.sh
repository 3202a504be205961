# Round-end evidence: GPU tests, smoke, bench (+CPU baseline), rocprof stats, B=32 bf16 / fp8 lines.
# usage: bash tools/gpu_round_end.sh <outdir-name>
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-full}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --kernel-steps 1 --no-cpu-baseline > $O/prof.log 2>&1
timeout -k 10 200 python bench.py --batch 32 --no-cpu-baseline > $O/bench_bf16_b32.json 2> $O/bench_bf16_b32.err
timeout -k 10 200 python bench.py --batch 32 --dtype fp8 --no-cpu-baseline > $O/bench_fp8_b32.json 2> $O/bench_fp8_b32.err
echo ALLDONE
