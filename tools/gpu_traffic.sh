# HBM traffic + SQ/MFMA counters of the resblock 3x3 conv family (fwd+stats / dgrad incl.
# the reflect ring / wgrad incl. its reduce) for bench.py's roofline.traffic: one
# rocprofv3 --pmc pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a
# pass; SQ groups within the 8-counter limit), then tools/traffic_summary.py.
# usage: bash tools/gpu_traffic.sh <outdir-name>
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-traffic}
mkdir -p $O
for K in fwd dgrad wgrad; do
  W=$K; [ $K = fwd ] && W=fwds
  MB="python tools/bench_conv.py --case res3x3_256@64 --iters 5 --which $W"
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$K -o run --output-format csv -- $MB > $O/fetch_$K.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write_$K -o run --output-format csv -- $MB > $O/write_$K.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq1_$K -o run --output-format csv -- $MB > $O/sq1_$K.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/sq2_$K -o run --output-format csv -- $MB > $O/sq2_$K.log 2>&1
done
python tools/traffic_summary.py $O > $O/traffic.json
cat $O/traffic.json

echo ALLDONE
