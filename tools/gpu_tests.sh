# GPU parity tests (all failures reported, per-test timeout).  usage: bash tools/gpu_tests.sh <outdir> [pytest args...]
export TMPDIR=/tmp
O=gpurun_out/${1:-tests}
shift || true
mkdir -p $O
timeout -k 10 1100 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread "${@:-tests}" > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -3 $O/pytest_gpu.log
echo ALLDONE
