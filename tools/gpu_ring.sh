# Conv/resample change check: kernel parity, conv microbench (wgrad split-K
# sweep, 256-wide wgrad tile), full GPU suite, bench, rocprof.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-ring}
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 60 --timeout-method thread > $O/pytest_kernels.log 2>&1
timeout -k 10 200 python tools/bench_conv.py --iters 20 --splitk 0,10,22,42 > $O/bench_conv.log 2>&1
IRGAN_WGH_256=1 timeout -k 10 100 python tools/bench_conv.py --iters 20 --case res3 --which wgrad --splitk 0,12,24 >> $O/bench_conv.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
echo ALLDONE
