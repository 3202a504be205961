# Round-6 pass y: MFMA head weight gradient -- full GPU suite, head kernels alone, step A/B (3 arms)
export TMPDIR=/tmp
O=gpurun_out/r06_y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest_gpu.txt)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" $O/pytest_gpu.txt | head -20; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_head -o run --output-format csv -- python3 tools/head_prof.py > $O/prof_head.log 2>&1 || { echo prof failed; exit 1; }
python tools/kernel_trace_summary.py $O/prof_head/run_kernel_trace.csv
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
