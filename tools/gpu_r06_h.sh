# Round-6 pass h: the ResnetBlock backward-data + IN backward-reduce fusion -- its tests, the
# related parity tests, then the step A/B (IRGAN_NO_DGRAD_INRED=1 = separate reduce pass),
# interleaved, and per-layer times with one stream
export TMPDIR=/tmp
O=gpurun_out/r06_h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dgrad_inred.py tests/test_gpu_ring_epi.py tests/test_gpu_step.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_on_$r.json 2> $O/bench_on_$r.err || { echo "on $r failed"; exit 1; }
  IRGAN_NO_DGRAD_INRED=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_off_$r.json 2> $O/bench_off_$r.err || { echo "off $r failed"; exit 1; }
done
python - <<PY
import json
for t in ("on", "off"):
    v = [json.load(open("$O/bench_%s_%d.json" % (t, r)))["value"] for r in (1, 2, 3)]
    print(t, v, "mean", round(sum(v) / 3, 1))
PY
IRGAN_NO_D_OVERLAP=1 timeout -k 10 300 python tools/layer_times.py > $O/layer_times_serial.txt 2>&1 || { echo lt failed; exit 1; }
grep -E "256x256k3s1r|in_bwd" $O/layer_times_serial.txt | head -12
echo ALLDONE
