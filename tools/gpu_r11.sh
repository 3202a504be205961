# wgrad wave-layout / split-K A/B on the resblock shape
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r11}
mkdir -p $O
timeout -k 10 120 python tools/bench_conv.py --iters 20 --case res3 --which wgrad --splitk 0,12,16,24,32 > $O/wg_base.log 2>&1
IRGAN_WGH_VAR=22 timeout -k 10 120 python tools/bench_conv.py --iters 20 --case res3 --which wgrad --splitk 0,12,16,24,32 > $O/wg_22.log 2>&1
IRGAN_WGH_VAR=14 timeout -k 10 120 python tools/bench_conv.py --iters 20 --case res3 --which wgrad --splitk 0,12,16,24,32 > $O/wg_14.log 2>&1
IRGAN_WGH_VAR=22 timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "conv_fwd_dgrad_wgrad" --timeout 60 --timeout-method thread > $O/pytest_22.log 2>&1
echo ALLDONE
