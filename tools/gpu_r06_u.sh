# Round-6 pass u: row-coalesced MaxPool2d backward (VGG pools) -- exactness tests, step A/B
# (IRGAN_NO_POOL_ROWS=1 = the per-pixel kernel), standalone times
export TMPDIR=/tmp
O=gpurun_out/r06_u; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16_elementwise.py tests/test_gpu_step.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
cat > $O/mp.py <<'PY'
import importlib, sys, torch
sys.path.insert(0, ".")
ops = importlib.import_module("infrared-colorization-with-resnet-generator-and-patchgan_amd").ops
for (N, H, C) in ((16, 256, 64), (16, 128, 128)):
    x = torch.relu(torch.randn(N, H, H, C, device="cuda")).bfloat16(); dy = torch.randn(N, H // 2, H // 2, C, device="cuda").bfloat16()
    dx = torch.empty_like(x)
    f = lambda: ops.maxpool_bwd(ops.Feat(x), ops.Feat(dy), ops.Feat(dx))
    for _ in range(3): f()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); a.record()
    for _ in range(20): f()
    b.record(); torch.cuda.synchronize()
    us = a.elapsed_time(b) / 20 * 1e3; by = x.numel() * 2 * 2 + dy.numel() * 2
    print(f"maxpool_bwd {N}x{H}x{H}x{C}: {us:.1f} us, {by / us / 1e3:.0f} GB/s", flush=True)
PY
timeout -k 10 120 python $O/mp.py > $O/mp_rows.txt 2>&1 && IRGAN_NO_POOL_ROWS=1 timeout -k 10 120 python $O/mp.py > $O/mp_old.txt 2>&1 || { echo mp failed; exit 1; }
echo rows; cat $O/mp_rows.txt; echo old; cat $O/mp_old.txt
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_on_$r.json 2>/dev/null || { echo "on $r failed"; exit 1; }
  IRGAN_NO_POOL_ROWS=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_off_$r.json 2>/dev/null || { echo "off $r failed"; exit 1; }
done
python - <<PY
import json
for t in ("on", "off"):
    v = [json.load(open("$O/bench_%s_%d.json" % (t, r)))["value"] for r in (1, 2, 3)]
    print(t, v, "mean", round(sum(v) / 3, 1))
PY
echo ALLDONE
