# resblock wgrad A/B: default (128-channel tile, 4 waves) vs IRGAN_WGH_256 (256-channel tile, 8 waves)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-wg256}
mkdir -p $O
timeout -k 10 120 python tools/bench_conv.py --iters 20 --case res3 --which wgrad --splitk 0,8,12,16,21 > $O/base.log 2>&1
IRGAN_WGH_256=1 timeout -k 10 120 python tools/bench_conv.py --iters 20 --case res3 --which wgrad --splitk 0,8,10,12,16,21 > $O/w256.log 2>&1
echo ALLDONE
