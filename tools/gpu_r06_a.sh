# Round-6 first GPU pass: full GPU suite, bench (256^2 B=16 and 512x640 B=4), conv_res64 ablations.
export TMPDIR=/tmp
O=gpurun_out/r06_a; mkdir -p $O
P=infrared-colorization-with-resnet-generator-and-patchgan_amd
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$? $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
echo "bench $(python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'])")"
timeout -k 10 300 python bench.py --height 512 --width 640 --batch 4 --no-cpu-baseline > $O/bench_512x640_b4.json 2> $O/bench_512.err || { echo bench512 failed; exit 1; }
echo "bench512 $(python -c "import json; d=json.load(open('$O/bench_512x640_b4.json')); print(d['value'], d['roofline']['frac'])")"
for v in default r64_nomfma r64_nostore r64_nohalo r64_nolds; do
  L=""; [ $v != default ] && L=$P/variants/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 200 python tools/bench_conv.py --case vgg12,vgg21,down1,up2,vgg22 --which fwd,fwds,dgrad,dgradm > $O/mb_$v.txt 2>&1 || { echo "mb $v failed"; exit 1; }
  echo "== $v"; grep "ms/TFLOPs" $O/mb_$v.txt
done
echo ALLDONE
