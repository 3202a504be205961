# Round-6 pass p: conv_pp epilogue cost, forward vs backward-data at the ResnetBlock shape
# (PP_EXP=16 variant: no epilogue), plus rocprof of the default microbench (interior vs ring)
export TMPDIR=/tmp
O=gpurun_out/r06_p; mkdir -p $O
B=infrared-colorization-with-resnet-generator-and-patchgan_amd/variants
for v in default pp_noepi default pp_noepi; do
  L=""; [ $v != default ] && L=$B/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 120 python tools/bench_conv.py --case res3x3_256@64 --which fwd,fwds,dgrad --iters 50 > $O/mb_$v.txt 2>&1 || { echo "$v failed"; tail -3 $O/mb_$v.txt; exit 1; }
  echo "$v: $(tail -1 $O/mb_$v.txt)"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python tools/bench_conv.py --case res3x3_256@64 --which fwd,fwds,dgrad --iters 20 > $O/prof.log 2>&1 || { echo prof failed; exit 1; }
python - <<PY
import csv
for r in csv.DictReader(open("$O/prof/run_kernel_stats.csv")):
    print(r["Name"][:110], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
echo ALLDONE
