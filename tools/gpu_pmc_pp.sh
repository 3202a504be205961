set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcpp}
mkdir -p $O
MB="python tools/bench_conv.py --case res3x3 --iters 3 --which fwd"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU -d $O/sq1 -o run --output-format csv -- $MB > $O/sq1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum -d $O/ta -o run --output-format csv -- $MB > $O/ta.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_LDS_WAVEFRONTS_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT -d $O/ta2 -o run --output-format csv -- $MB > $O/ta2.log 2>&1
echo ALLDONE
