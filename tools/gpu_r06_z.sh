# Round-6 pass z: PatchGAN head forward in one launch (Z in LDS) vs two launches -- tests, kernels
# alone (both), step A/B (interleaved x3)
export TMPDIR=/tmp
O=gpurun_out/r06_z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_patch_head.py tests/test_gpu_step.py tests/test_gpu_module_api.py tests/test_gpu_bf16_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
IRGAN_HEAD_FWD_FUSED=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_patch_head.py tests/test_gpu_step.py -x -q --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1
rc=$?; echo "pytest fused rc=$rc $(tail -1 $O/pytest_fused.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest_fused.log | head -20; exit 1; }
IRGAN_HEAD_FWD_FUSED=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_fused -o run --output-format csv -- python3 tools/head_prof.py > $O/prof_fused.log 2>&1 || { echo prof failed; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_split -o run --output-format csv -- python3 tools/head_prof.py > $O/prof_split.log 2>&1 || { echo prof2 failed; exit 1; }
python tools/kernel_trace_summary.py $O/prof_fused/run_kernel_trace.csv $O/prof_split/run_kernel_trace.csv
for r in 1 2 3; do
  IRGAN_HEAD_FWD_FUSED=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fused_$r.json 2>/dev/null || { echo "fused $r failed"; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_split_$r.json 2>/dev/null || { echo "split $r failed"; exit 1; }
done
python - <<PY
import json
for t in ("fused", "split"):
    v = [json.load(open("$O/bench_%s_%d.json" % (t, r)))["value"] for r in (1, 2, 3)]
    print(t, v, "mean", round(sum(v) / 3, 1))
PY
echo ALLDONE
