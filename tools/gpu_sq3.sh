# SQ MFMA-busy / GRBM passes for the resblock conv family, one pass per family.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-sq3}
mkdir -p $O
for K in fwd dgrad wgrad; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/$K -o run --output-format csv -- python tools/bench_conv.py --case res3x3 --iters 5 --which $K > $O/$K.log 2>&1
done
echo ALLDONE
