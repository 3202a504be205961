# One iteration pass: the GPU suite (tests, smoke, bench), the narrow-conv microbench, then
# same-box A/B of variant libraries for the resblock convs and the InstanceNorm passes.
# usage: bash tools/gpu_iter.sh <name> "<conv variants>" "<norm variants>"
export TMPDIR=/tmp
N=${1:-iter}
bash tools/gpu_suite.sh $N || exit 1
timeout -k 10 120 python tools/c8_bench.py > gpurun_out/$N/c8.txt 2>&1 || { echo "c8 bench failed"; tail -3 gpurun_out/$N/c8.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/$N/c8.txt
if [ -n "$2" ]; then bash tools/gpu_libab.sh ${N}_ab "--case res3x3 --which fwds,dgrad,wgrad" "" $2 || exit 1; fi
if [ -n "$3" ]; then bash tools/gpu_normab.sh ${N}_nab $3 || exit 1; fi
echo ITER_DONE
