# pp128 (Cout 128 ping-pong conv): parity, conv microbench A/B, full suite, default bench (with CPU baseline), rocprof
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r7}
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 60 --timeout-method thread > $O/pytest_kernels.log 2>&1
timeout -k 10 150 python tools/bench_conv.py --iters 20 --which fwd,dgrad > $O/bench_conv.log 2>&1
IRGAN_NO_PP128=1 timeout -k 10 150 python tools/bench_conv.py --iters 20 --which fwd,dgrad > $O/bench_conv_old.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
echo ALLDONE
