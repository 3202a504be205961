# Round-6 pass m: W2 A/B -- s_setprio 1 on the compute waves (W2_EXP=16 variant)
export TMPDIR=/tmp
O=gpurun_out/r06_m; mkdir -p $O
B=infrared-colorization-with-resnet-generator-and-patchgan_amd/variants
for v in default w2_prio default w2_prio; do
  L=""; [ $v != default ] && L=$B/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 120 python tools/bench_conv.py --case res3x3_256@64 --which wgrad --iters 50 > $O/mb_$v.txt 2>&1 || { echo "$v failed"; exit 1; }
  echo "$v: $(tail -1 $O/mb_$v.txt)"
done
echo ALLDONE
