# pp192 / pp64 candidates: parity with each on, conv microbench A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r8}
mkdir -p $O
IRGAN_PP192=1 IRGAN_PP64=1 timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 60 --timeout-method thread > $O/pytest_kernels.log 2>&1
timeout -k 10 150 python tools/bench_conv.py --iters 20 --which fwd,dgrad --case @256 > $O/bench_conv_base.log 2>&1
IRGAN_PP192=1 timeout -k 10 150 python tools/bench_conv.py --iters 20 --which fwd,dgrad --case @256 > $O/bench_conv_192.log 2>&1
IRGAN_PP64=1 timeout -k 10 150 python tools/bench_conv.py --iters 20 --which fwd,dgrad --case @256 > $O/bench_conv_64.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_base.json 2> $O/bench.err
IRGAN_PP192=1 IRGAN_PP64=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_both.json 2>> $O/bench.err
IRGAN_PP192=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_192.json 2>> $O/bench.err
echo ALLDONE
