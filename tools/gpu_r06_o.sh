# Round-6 pass o: the MFMA probe (test + bench's measured peak)
export TMPDIR=/tmp
O=gpurun_out/r06_o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k mfma_probe -x -v -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(grep 'measured bf16' $O/pytest.log) $(tail -1 $O/pytest.log)"
[ $rc -ne 0 ] && { tail -20 $O/pytest.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -5 $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --batch 32 --dtype fp8 --no-cpu-baseline > $O/bench_fp8.json 2> $O/bench_fp8.err || { echo bench fp8 failed; exit 1; }
python - <<PY
import json
for f in ("bench", "bench_fp8"):
    d = json.load(open("$O/%s.json" % f)); r = d["roofline"]
    print(f, d["value"], r["kernel"], r["achieved"], r["peak"], r["frac"], r["peak_measured"], r["frac_of_measured_peak"])
PY
echo ALLDONE
