# Round-6 pass j: the fp8 step outside the fp8 kernels' limits, then pass i
# (W2 ablations)
export TMPDIR=/tmp
O=gpurun_out/r06_j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py -k beyond -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
bash tools/gpu_r06_i.sh
