set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/p7
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -q -x > gpurun_out/p7/pytest_kernels.log 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_step.py tests/test_integration_stub.py -q -x > gpurun_out/p7/pytest_step.log 2>&1
timeout -k 10 200 python tools/bench_conv.py --iters 20 > gpurun_out/p7/bench_conv.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/p7/bench.json 2> gpurun_out/p7/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p7/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/p7/prof.log 2>&1
echo ALLDONE
