# DP overlap check: step parity tests, 2-rank gloo DP test on one GPU, bench
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-dp}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_step.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo ALLDONE
