# PMC passes (HBM bytes + SQ wait / MFMA counters) for the 64-channel 256^2 / 128^2 conv family
# (down1 forward + IN statistics, VGG conv1_2 / conv2_1 forward, up2_conv
# forward / backward-data / weight gradient), one rocprofv3 --pmc pass per counter group per
# case over tools/bench_conv.py, then tools/traffic_c64.py.  usage: bash tools/gpu_pmc_c64.sh <outdir-name>
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_c64}
mkdir -p $O
for C in "down1:fwds" "down1:fwd" "vgg12:fwd" "vgg21:fwd" "up2:fwds" "up2:dgrad" "up2:wgrad"; do
  CASE=${C%%:*}; W=${C##*:}; T=${CASE}_$W
  MB="python tools/bench_conv.py --case $CASE --iters 5 --which $W"
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$T -o run --output-format csv -- $MB > $O/fetch_$T.log 2>&1 || { echo "pmc failed $T"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write_$T -o run --output-format csv -- $MB > $O/write_$T.log 2>&1 || { echo "pmc failed $T"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq1_$T -o run --output-format csv -- $MB > $O/sq1_$T.log 2>&1 || { echo "pmc failed $T"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/sq2_$T -o run --output-format csv -- $MB > $O/sq2_$T.log 2>&1 || { echo "pmc failed $T"; exit 1; }
  echo "done $T"
done
python tools/traffic_c64.py $O > $O/pmc_c64.json && cat $O/pmc_c64.json
echo ALLDONE
