# PMC passes (one counter group per rocprofv3 run) over (a) the resblock conv
# microbench and (b) a short bench.py run for per-dispatch HBM traffic.
# usage: bash tools/gpu_pmc.sh <outdir-name>
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc}
mkdir -p $O
MB="python tools/bench_conv.py --case res3x3 --iters 3"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq1 -o run --output-format csv -- $MB > $O/sq1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/sq2 -o run --output-format csv -- $MB > $O/sq2.log 2>&1 || echo "sq2 failed" >> $O/sq2.log
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_mb -o run --output-format csv -- $MB > $O/fetch_mb.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write_mb -o run --output-format csv -- $MB > $O/write_mb.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_bench -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/fetch_bench.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/write_bench -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/write_bench.log 2>&1
echo ALLDONE
