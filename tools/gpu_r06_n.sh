# Round-6 pass n: W3 weight gradient (IRGAN_W3=1) -- bit identity against W2 on fixed operands,
# the wgrad parity tests and the step under W3, microbench and step A/B
export TMPDIR=/tmp
O=gpurun_out/r06_n; mkdir -p $O
timeout -k 10 120 python tools/w3_check.py $O/w2.pt > $O/w2.txt 2>&1 || { echo w2 check failed; cat $O/w2.txt | tail -3; exit 1; }
IRGAN_W3=1 timeout -k 10 120 python tools/w3_check.py $O/w3.pt > $O/w3.txt 2>&1 || { echo w3 check failed; tail -3 $O/w3.txt; exit 1; }
python - <<PY
import torch
a, b = torch.load("$O/w2.pt"), torch.load("$O/w3.pt")
for k in a:
    print(k, "bit-identical" if torch.equal(a[k], b[k]) else "DIFFER max %g" % (a[k] - b[k]).abs().max())
PY
IRGAN_W3=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16_parity.py tests/test_gpu_step.py -x -q --timeout 300 --timeout-method thread > $O/pytest_w3.log 2>&1
rc=$?; echo "pytest (W3) rc=$rc $(tail -1 $O/pytest_w3.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest_w3.log | head; exit 1; }
for v in 0 1 0 1; do
  IRGAN_W3=$v timeout -k 10 120 python tools/bench_conv.py --case res3x3_256@64,res3x3_256@128x160b4 --which wgrad --iters 50 > $O/mb_$v.txt 2>&1 || { echo "mb $v failed"; exit 1; }
  echo "W3=$v: $(tail -2 $O/mb_$v.txt | tr '\n' ' ')"
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_w2_$r.json 2>/dev/null || { echo bench failed; exit 1; }
  IRGAN_W3=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_w3_$r.json 2>/dev/null || { echo bench w3 failed; exit 1; }
done
python - <<PY
import json
for t in ("w2", "w3"):
    print(t, [json.load(open("$O/bench_%s_%d.json" % (t, r)))["value"] for r in (1, 2)])
PY
echo ALLDONE
