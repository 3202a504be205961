# Round-6 pass c: same-box A/B of the res64 run statistics and the VGG conv+pool fusion,
# conv microbench incl. the BN round model at 128 x 160, and a kernel trace of the step.
export TMPDIR=/tmp
O=gpurun_out/r06_c; mkdir -p $O
P=infrared-colorization-with-resnet-generator-and-patchgan_amd
timeout -k 10 200 python tools/bench_conv.py --case vgg12,down1,res3x3_256@128x160b4 --which fwd,fwds,dgrad,wgrad > $O/mb_default.txt 2>&1 || { echo "mb failed"; exit 1; }
echo "== default"; grep "ms/TFLOPs" $O/mb_default.txt
IRGAN_R64_PATCH_STATS=1 timeout -k 10 200 python tools/bench_conv.py --case vgg12,down1 --which fwds > $O/mb_patchstats.txt 2>&1 || { echo "mb2 failed"; exit 1; }
echo "== per-patch stats"; grep "ms/TFLOPs" $O/mb_patchstats.txt
IRGAN_LIB=$P/variants/libirgan_bn_old.so timeout -k 10 200 python tools/bench_conv.py --case res3x3_256@128x160b4 --which fwd,fwds,dgrad > $O/mb_bnold.txt 2>&1 || { echo "mb3 failed"; exit 1; }
echo "== bn old"; grep "ms/TFLOPs" $O/mb_bnold.txt
for rep in 1 2; do
  for envs in "IRGAN_NONE=1" "IRGAN_R64_PATCH_STATS=1" "IRGAN_NO_POOL_FUSION=1" "IRGAN_R64_PATCH_STATS=1 IRGAN_NO_POOL_FUSION=1"; do
    tag=$(echo $envs | tr ' =' '__')
    timeout -k 10 300 env $envs python bench.py --no-cpu-baseline > $O/bench_${tag}_$rep.json 2> $O/bench_${tag}_$rep.err || { echo "bench $envs failed"; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${tag}_$rep.json')); print('$envs', d['value'], d['ms_per_step_median'])"
  done
done
IRGAN_LIB=$P/variants/libirgan_bn_old.so timeout -k 10 300 python bench.py --height 512 --width 640 --batch 4 --no-cpu-baseline > $O/bench_512_bnold.json 2> $O/bench_512_bnold.err || { echo bench512old failed; exit 1; }
echo "bench512 bnold $(python -c "import json; d=json.load(open('$O/bench_512_bnold.json')); print(d['value'], d['ms_per_step_median'], {k: v['mean_ms'] for k, v in d['roofline']['per_kernel'].items()})")"
timeout -k 10 300 python bench.py --height 512 --width 640 --batch 4 --no-cpu-baseline > $O/bench_512.json 2> $O/bench_512.err || { echo bench512 failed; exit 1; }
echo "bench512 $(python -c "import json; d=json.load(open('$O/bench_512.json')); print(d['value'], d['ms_per_step_median'], {k: v['mean_ms'] for k, v in d['roofline']['per_kernel'].items()})")"
bash tools/gpu_trace.sh r06_c/trace
echo ALLDONE
