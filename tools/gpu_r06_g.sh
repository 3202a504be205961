# Round-6 pass g: full GPU suite + smoke on the current tree, per-layer times in the step and
# with one stream (IRGAN_NO_D_OVERLAP=1: each launch alone on the GPU)
export TMPDIR=/tmp
O=gpurun_out/r06_g; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -rP --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest_gpu.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED" $O/pytest_gpu.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$? $(tail -1 $O/smoke.log)"
timeout -k 10 300 python tools/layer_times.py > $O/layer_times.txt 2>&1 || { echo lt failed; exit 1; }
IRGAN_NO_D_OVERLAP=1 timeout -k 10 300 python tools/layer_times.py > $O/layer_times_serial.txt 2>&1 || { echo lt2 failed; exit 1; }
head -45 $O/layer_times_serial.txt
echo ALLDONE
