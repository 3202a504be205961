# Round-6 pass i: W2 weight-gradient ablations (W2_EXP variants of conv_wgrad_pc.hip) at the
# ResnetBlock shape (B = 16, 64x64, 256 -> 256), microbench incl. the split-K reduce
export TMPDIR=/tmp
O=gpurun_out/r06_i; mkdir -p $O
B=infrared-colorization-with-resnet-generator-and-patchgan_amd/variants
for v in default w2_nostore w2_nodma w2_nomfma default; do
  L=""; [ $v != default ] && L=$B/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 120 python tools/bench_conv.py --case res3x3_256@64 --which wgrad --iters 50 > $O/mb_$v.txt 2>&1 || { echo "$v failed"; exit 1; }
  echo "$v: $(tail -1 $O/mb_$v.txt)"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/bench_conv.py --case res3x3_256@64 --which wgrad --iters 20 > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
grep -E "wgrad" $O/prof/run_kernel_stats.csv | cut -c1-160
echo ALLDONE
