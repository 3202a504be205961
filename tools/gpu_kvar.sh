# per-kernel times of one conv microbench case under variant libraries (rocprofv3 --stats):
# usage: bash tools/gpu_kvar.sh <outdir> "<bench_conv.py args>" <variant> [<variant> ...]
export TMPDIR=/tmp
O=gpurun_out/$1; shift
MB=$1; shift
mkdir -p $O
B=infrared-colorization-with-resnet-generator-and-patchgan_amd/variants
for v in default "$@"; do
  L=""; [ $v != default ] && L=$B/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_$v -o run --output-format csv -- python tools/bench_conv.py $MB > $O/mb_$v.txt 2>&1 || { echo "variant $v failed"; tail -3 $O/mb_$v.txt; exit 1; }
  S=$(find $O/p_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v: $(tail -1 $O/mb_$v.txt)"
  python -c "
import csv,sys
for r in csv.DictReader(open('$S')):
    n=r['Name'].replace('(anonymous namespace)::','').split('(')[0][:60]
    if 'at::' in n: continue
    print(f\"   {float(r['AverageNs'])/1e3:8.1f} us x {r['Calls']:>4}  {n}\")
"
done
echo ALLDONE
