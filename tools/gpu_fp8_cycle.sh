# fp8 kernel + step tests, then the config-5 bench lines.  usage: bash tools/gpu_fp8_cycle.sh <outdir-name>
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-fp8}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_fp8.py -s > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --batch 32 --dtype fp8 --steps 20 --no-cpu-baseline > $O/bench_fp8.json 2> $O/bench_fp8.err
echo ALLDONE
