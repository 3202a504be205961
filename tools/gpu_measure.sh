# Measurement pass: step profile (tools/gpu_profile.sh), conv microbenchmarks of the layers
# under work, and the PMC traffic / MFMA counters of the resblock family (tools/gpu_traffic.sh).
# usage: bash tools/gpu_measure.sh <outdir-name>
export TMPDIR=/tmp
N=${1:-measure}
O=gpurun_out/$N
mkdir -p $O
bash tools/gpu_profile.sh $N/profile || exit 1
MB="timeout -k 10 120 python tools/bench_conv.py --iters 20"
$MB --case res3x3 --which fwds,dgrad,wgrad > $O/mb_res.txt 2>&1 || { echo "mb res failed"; tail -3 $O/mb_res.txt; exit 1; }
$MB --case vgg --which fwdr,dgradm,wgrad > $O/mb_vgg.txt 2>&1 || { echo "mb vgg failed"; tail -3 $O/mb_vgg.txt; exit 1; }
$MB --case D --batch 32 --which fwd,dgrad,wgrad > $O/mb_d32.txt 2>&1 || { echo "mb D failed"; tail -3 $O/mb_d32.txt; exit 1; }
grep "ms/TFLOPs" $O/mb_*.txt
bash tools/gpu_traffic.sh $N/pmc > $O/traffic.log 2>&1 || { echo "traffic failed"; tail -5 $O/traffic.log; exit 1; }
tail -40 $O/pmc/traffic.json
echo ALLDONE
