# kernel parity, HBM microbench (rows8 on / off), full GPU suite, bench, rocprof
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r3}
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 60 --timeout-method thread > $O/pytest_kernels.log 2>&1
timeout -k 10 120 python tools/bench_hbm.py --case @ > $O/hbm.log 2>&1
IRGAN_NO_ROWS8=1 timeout -k 10 120 python tools/bench_hbm.py --case @ > $O/hbm_old.log 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
echo ALLDONE
