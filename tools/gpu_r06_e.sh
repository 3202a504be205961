# Round-6 pass e: full GPU suite, bench lines (B=16 bf16, B=32 bf16 / fp8), 64-channel family PMC
export TMPDIR=/tmp
O=gpurun_out/r06_e; mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -rP --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest_gpu.log)"
[ $rc -ne 0 ] && grep -E "^FAILED" $O/pytest_gpu.log | head
grep -E "fp8 ResnetBlock dW at|vs fp32:|loss_G first-20" $O/pytest_gpu.log | head
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
echo "bench $(python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step_median'], d['roofline']['frac'])")"
timeout -k 10 300 python bench.py --batch 32 --no-cpu-baseline > $O/bench_bf16_b32.json 2> $O/bench_bf16_b32.err || { echo bench32 failed; exit 1; }
timeout -k 10 300 python bench.py --batch 32 --dtype fp8 --no-cpu-baseline > $O/bench_fp8_b32.json 2> $O/bench_fp8_b32.err || { echo bench fp8 failed; exit 1; }
echo "b32 bf16 / fp8 $(python -c "import json; a=json.load(open('$O/bench_bf16_b32.json')); b=json.load(open('$O/bench_fp8_b32.json')); print(a['value'], b['value'], round(b['value']/a['value']-1, 4))")"
bash tools/gpu_pmc_c64.sh r06_e/pmc_c64 > $O/pmc.log 2>&1; echo "pmc rc=$?"; tail -3 $O/pmc.log
echo ALLDONE
