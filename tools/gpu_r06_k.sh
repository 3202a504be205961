# Round-6 pass k: full GPU suite + smoke on the current tree (library rebuilt after the revert)
export TMPDIR=/tmp
O=gpurun_out/r06_k; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -rP --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest_gpu.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED" $O/pytest_gpu.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$? $(tail -1 $O/smoke.log)"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step_median'], d['roofline']['frac'])"
echo ALLDONE
