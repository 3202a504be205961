# wgrad slab vs atomics (conv microbench A/B), kernel parity, full GPU suite, bench, rocprof
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r4}
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 60 --timeout-method thread > $O/pytest_kernels.log 2>&1
timeout -k 10 150 python tools/bench_conv.py --iters 20 --which wgrad > $O/bench_conv.log 2>&1
IRGAN_NO_WGRAD_SLAB=1 timeout -k 10 150 python tools/bench_conv.py --iters 20 --which wgrad > $O/bench_conv_atomic.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
echo ALLDONE
