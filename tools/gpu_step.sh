# step-level GPU tests only
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-step}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
echo ALLDONE
