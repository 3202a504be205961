# Round-6 pass x: PatchGAN head on MFMA (fwd tap GEMM + sum, dgrad hi/lo GEMM) + VALU wgrad
# -- tests, D / step parity, layer times, step A/B (3 arms, interleaved)
export TMPDIR=/tmp
O=gpurun_out/r06_x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_patch_head.py tests/test_gpu_step.py tests/test_gpu_module_api.py tests/test_gpu_bf16_parity.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
IRGAN_NO_D_OVERLAP=1 timeout -k 10 300 python tools/layer_times.py > $O/layer_times_serial.txt 2>&1 || { echo lt failed; exit 1; }
grep -E "512x1k4" $O/layer_times_serial.txt
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_on_$r.json 2>/dev/null || { echo "on $r failed"; exit 1; }
  IRGAN_NO_HEAD_WGRAD=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_nowg_$r.json 2>/dev/null || { echo "nowg $r failed"; exit 1; }
  IRGAN_NO_PATCH_HEAD=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_off_$r.json 2>/dev/null || { echo "off $r failed"; exit 1; }
done
python - <<PY
import json
for t in ("on", "nowg", "off"):
    v = [json.load(open("$O/bench_%s_%d.json" % (t, r)))["value"] for r in (1, 2, 3)]
    print(t, v, "mean", round(sum(v) / 3, 1))
PY
echo ALLDONE
