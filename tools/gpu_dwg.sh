# D small-spatial wgrad split-K sweep (conv_wgrad_glds)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-dwg}
mkdir -p $O
timeout -k 10 120 python tools/bench_conv.py --iters 20 --case D --which wgrad --splitk 0,1,2,8,16,32,64 > $O/dwg.log 2>&1
echo ALLDONE
