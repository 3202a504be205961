# round-4 wgrad experiments: fp8 weight gradient parity, wide-n bf16 wgrad parity + microbench
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_c}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -q -x --timeout 120 --timeout-method thread -k "wgrad" > $O/t_fp8w.log 2>&1
rc=$?; echo "fp8 wgrad tests rc=$rc"; tail -2 $O/t_fp8w.log
[ $rc -le 1 ] && ! grep -q "+ Timeout +" $O/t_fp8w.log || exit 1   # a test failure goes on; a fault / abort / time limit ends the script
IRGAN_WGRAD_W2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16_parity.py -q -x --timeout 120 --timeout-method thread -k "family" > $O/t_w2.log 2>&1 || { echo "w2 parity failed"; tail -5 $O/t_w2.log; exit 1; }
tail -1 $O/t_w2.log
for e in "" "IRGAN_WGRAD_W2=1"; do
  env $e timeout -k 10 120 python tools/bench_conv.py --case res3x3 --which wgrad --iters 50 > $O/mb_$e.txt 2>&1 || exit 1
  echo "wgrad [$e]: $(tail -1 $O/mb_$e.txt)"
done
timeout -k 10 120 python tools/fp8_bench.py > $O/fp8_bench.txt 2>&1 && tail -5 $O/fp8_bench.txt
echo ALLDONE
