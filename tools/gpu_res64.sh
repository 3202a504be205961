# res64 kernel: bf16 parity tests, conv microbench A/B (IRGAN_NO_RES64), step bench.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-res64}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_bf16.log 2>&1
for E in "-" "IRGAN_NO_RES64=1"; do
  echo "## $E" >> $O/ab.txt
  if [ "$E" = "-" ]; then E=""; fi
  env $E timeout -k 10 120 python tools/bench_conv.py --case 64 --which fwd,fwds,dgrad >> $O/ab.txt 2>&1
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo ALLDONE
