# SQ counter passes over the conv microbench (one rocprofv3 --pmc pass per group).
# usage: bash tools/gpu_sq.sh <outdir-name> "<bench_conv.py args>"
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-sq}
ARGS=${2:---case res3x3 --iters 3}
mkdir -p $O
MB="python tools/bench_conv.py $ARGS"
timeout -k 10 120 $MB > $O/plain.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq1 -o run --output-format csv -- $MB > $O/sq1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/sq2 -o run --output-format csv -- $MB > $O/sq2.log 2>&1
echo ALLDONE
