# config-4 shape test + PMC traffic re-measure (wgrad now slab-reduced)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r6}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -x -v -k 512x640 --timeout 240 --timeout-method thread > $O/pytest_512.log 2>&1
bash tools/gpu_traffic.sh ${1:-r6}/traffic
echo ALLDONE
