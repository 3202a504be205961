# GPU parity tests only.  usage: bash tools/gpu_tests.sh <outdir-name> [pytest args...]
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-tests}
shift || true
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "${@:-tests}" > $O/pytest_gpu.log 2>&1
echo ALLDONE
