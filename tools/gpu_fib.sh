# Fused IN-backward reduce (opt-in): its GPU tests, then the step A/B (default vs IRGAN_FUSED_IN_BWD=1).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r02_fib
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused_in_bwd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_fib/t1.log 2>&1
bash tools/gpu_ab_bench.sh r02_fib "-" "IRGAN_FUSED_IN_BWD=1"
