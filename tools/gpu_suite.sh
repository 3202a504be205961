# Full GPU suite (no -x: every failure is listed), then smoke and the default bench line.
# Stops after a crash/timeout (rc other than 0/1 from pytest) -- nothing more runs on the GPU.
# usage: bash tools/gpu_suite.sh <outdir-name>
export TMPDIR=/tmp
O=gpurun_out/${1:-suite}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
echo "pytest rc=$rc"
