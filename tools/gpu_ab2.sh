# Round-5 iteration pass: the GPU suite (tests, smoke, bench), the D-layer and resblock conv
# microbenchmarks, and the step phases.  usage: bash tools/gpu_ab2.sh <outdir-name>
export TMPDIR=/tmp
N=${1:-iter}
O=gpurun_out/$N
mkdir -p $O
bash tools/gpu_suite.sh $N || exit 1
MB="timeout -k 10 120 python tools/bench_conv.py --iters 20"
$MB --case D --batch 32 --which fwd,dgrad,wgrad > $O/mb_d32.txt 2>&1 || { echo "mb D failed"; tail -3 $O/mb_d32.txt; exit 1; }
$MB --case res3x3 --which fwds,dgrad,wgrad > $O/mb_res.txt 2>&1 || { echo "mb res failed"; exit 1; }
grep "ms/TFLOPs" $O/mb_*.txt
bash tools/gpu_phases.sh $N/ph || exit 1
IRGAN_NO_D_OVERLAP=1 timeout -k 10 200 python tools/layer_times.py > $O/layers_serial.txt 2>&1 || exit 1
grep -E "4s2z|512x1" $O/layers_serial.txt
echo ALLDONE
