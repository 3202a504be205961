# round-4: fp8 weight gradient in the step (tight + step tests), wide-n bf16 wgrad default
# (parity), host-enqueue trace of the bf16 step, config-5 bench fp8 vs bf16 at B=32
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_d}
mkdir -p $O
T="python -u -m pytest -q -x --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_fp8.py > $O/t_fp8.log 2>&1
rc=$?; echo "fp8 tests rc=$rc"; tail -3 $O/t_fp8.log
[ $rc -le 1 ] && ! grep -q "+ Timeout +" $O/t_fp8.log || exit 1
timeout -k 10 400 $T tests/test_gpu_bf16_parity.py > $O/t_bf16.log 2>&1 || { echo "bf16 parity failed"; tail -5 $O/t_bf16.log; exit 1; }
tail -1 $O/t_bf16.log
bash tools/gpu_apitrace.sh ${1:-r04_d}/api || exit 1
for a in "--batch 16 --dtype bf16" "--batch 32 --dtype bf16" "--batch 32 --dtype fp8"; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline $a > $O/bench.txt 2>&1 || { tail -5 $O/bench.txt; exit 1; }
  echo "[$a] $(tail -1 $O/bench.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
echo ALLDONE
