# Round-6 pass f: the pipelined resample (sep_pipe_kernel) -- tests, microbench vs the one-row
# kernel (IRGAN_SEP_ROWS1=1), step A/B
export TMPDIR=/tmp
O=gpurun_out/r06_f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16_elementwise.py tests/test_gpu_fp8.py tests/test_gpu_step.py \
  tests/test_gpu_kernels.py tests/test_gpu_module_api.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest_gpu.log)"
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
timeout -k 10 120 python tools/resample_bench.py > $O/rs_new.txt 2>&1 && IRGAN_SEP_ROWS1=1 timeout -k 10 120 python tools/resample_bench.py > $O/rs_old.txt 2>&1 || { echo rsbench failed; exit 1; }
echo "== new"; grep " us " $O/rs_new.txt; echo "== old"; grep " us " $O/rs_old.txt
for rep in 1 2 3; do
  for envs in "IRGAN_NONE=1" "IRGAN_SEP_ROWS1=1"; do
    tag=$(echo $envs | tr ' =' '__')
    timeout -k 10 300 env $envs python bench.py --no-cpu-baseline > $O/bench_${tag}_$rep.json 2> $O/bench_${tag}_$rep.err || { echo "bench $envs failed"; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${tag}_$rep.json')); print('$envs', d['value'], d['ms_per_step_median'])"
  done
done
echo ALLDONE
