set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r02_xcdg
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_parity.py -x -q -k "res64 or 64" --timeout 200 --timeout-method thread > gpurun_out/r02_xcdg/t.log 2>&1
for r in 1 2; do for E in IRGAN_RES64_NO_XCDG=1 IRGAN_DUMMY=1; do echo "## $E"; env $E timeout -k 10 100 python tools/bench_conv.py --case 64 --which fwd,fwds,dgrad; done; done
bash tools/gpu_ab_bench.sh r02_xcdg "-" "IRGAN_RES64_NO_XCDG=1"
