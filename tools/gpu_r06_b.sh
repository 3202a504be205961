# Round-6 second GPU pass: targeted GPU tests, bench (256^2 B=16, 512x640 B=4), conv microbench
# (res64 stats runs vs per-patch, the BN round model vs the round-5 rule at 128 x 160).
export TMPDIR=/tmp
O=gpurun_out/r06_b; mkdir -p $O
P=infrared-colorization-with-resnet-generator-and-patchgan_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16_parity.py tests/test_gpu_fp8.py tests/test_gpu_trajectory.py \
  tests/test_gpu_dp.py tests/test_gpu_kernels.py tests/test_gpu_step.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$? $(tail -1 $O/pytest_gpu.log)"
grep -E "fp8 dW at|worst rel-L2|vs fp32:|loss_G first-20" $O/pytest_gpu.log | head -20
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
echo "bench $(python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step_median'], d['roofline']['frac'])")"
timeout -k 10 300 python bench.py --height 512 --width 640 --batch 4 --no-cpu-baseline > $O/bench_512x640_b4.json 2> $O/bench_512.err || { echo bench512 failed; exit 1; }
echo "bench512 $(python -c "import json; d=json.load(open('$O/bench_512x640_b4.json')); print(d['value'], d['ms_per_step_median'], {k: v['mean_ms'] for k, v in d['roofline']['per_kernel'].items()})")"
timeout -k 10 200 python tools/bench_conv.py --case vgg12,down1,up2,res3x3_256@128x160b4 --which fwd,fwds,dgrad,dgradm,wgrad > $O/mb_default.txt 2>&1 || { echo "mb failed"; exit 1; }
echo "== default"; grep "ms/TFLOPs" $O/mb_default.txt
IRGAN_R64_PATCH_STATS=1 timeout -k 10 200 python tools/bench_conv.py --case vgg12,down1 --which fwds > $O/mb_patchstats.txt 2>&1 || { echo "mb2 failed"; exit 1; }
echo "== per-patch stats"; grep "ms/TFLOPs" $O/mb_patchstats.txt
IRGAN_LIB=$P/variants/libirgan_bn_old.so timeout -k 10 200 python tools/bench_conv.py --case res3x3_256@128x160b4 --which fwd,fwds,dgrad > $O/mb_bnold.txt 2>&1 || { echo "mb3 failed"; exit 1; }
echo "== bn old"; grep "ms/TFLOPs" $O/mb_bnold.txt
IRGAN_LIB=$P/variants/libirgan_bn_old.so timeout -k 10 300 python bench.py --height 512 --width 640 --batch 4 --no-cpu-baseline > $O/bench_512_bnold.json 2> $O/bench_512_bnold.err || { echo bench512old failed; exit 1; }
echo "bench512 bnold $(python -c "import json; d=json.load(open('$O/bench_512_bnold.json')); print(d['value'], d['ms_per_step_median'], {k: v['mean_ms'] for k, v in d['roofline']['per_kernel'].items()})")"
echo ALLDONE
