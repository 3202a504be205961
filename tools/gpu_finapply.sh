set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r02_finapp
timeout -k 10 200 python -u -m pytest tests/test_gpu_fin_apply.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_finapp/t1.log 2>&1
bash tools/gpu_ab_bench.sh r02_finapp "-" "IRGAN_NO_FIN_APPLY=1"
