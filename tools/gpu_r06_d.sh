# Round-6 pass d: targeted GPU tests, then a same-box A/B: D weight gradients on the main
# stream vs all on the side stream, the VGG conv+pool fusion (now DPP) on / off.
export TMPDIR=/tmp
O=gpurun_out/r06_d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16_parity.py tests/test_gpu_dp.py tests/test_gpu_step.py tests/test_gpu_kernels.py tests/test_gpu_module_variants.py tests/test_gpu_eval.py \
  tests/test_gpu_module_api.py -m gpu -x -q -rP --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$? $(tail -1 $O/pytest_gpu.log)"
[ $? -ne 0 ] && grep -E "FAILED|Error" $O/pytest_gpu.log | head
timeout -k 10 200 python tools/bench_conv.py --case vgg12,down1 --which fwd,fwds > $O/mb_default.txt 2>&1 || { echo "mb failed"; exit 1; }
grep "ms/TFLOPs" $O/mb_default.txt
for rep in 1 2 3; do
  for envs in "IRGAN_NONE=1" "IRGAN_D_WGRAD_SIDE=1" "IRGAN_NO_POOL_FUSION=1"; do
    tag=$(echo $envs | tr ' =' '__')
    IRGAN_JOIN_TIMING=1 timeout -k 10 300 env $envs python bench.py --no-cpu-baseline > $O/bench_${tag}_$rep.json 2> $O/bench_${tag}_$rep.err || { echo "bench $envs failed"; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${tag}_$rep.json')); print('$envs', d['value'], d['ms_per_step_median'], 'join_wait', d.get('join_wait_ms'), d.get('step_phase_ms'))"
  done
done
echo ALLDONE
