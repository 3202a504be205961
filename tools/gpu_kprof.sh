# Per-kernel times of one conv microbenchmark under rocprofv3 for the default library and
# variant builds (tools/build_variant.sh), e.g. the ring line GEMM's ablations (RING_EXP).
# usage: bash tools/gpu_kprof.sh <outdir> "<bench_conv.py args>" <variant> [<variant> ...]
export TMPDIR=/tmp
O=gpurun_out/$1; shift
MB=$1; shift
mkdir -p $O
B=infrared-colorization-with-resnet-generator-and-patchgan_amd/variants
for v in default "$@"; do
  L=""; [ $v != default ] && L=$B/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_$v -o run --output-format csv -- python tools/bench_conv.py $MB > $O/mb_$v.txt 2>&1 || { echo "$v failed"; tail -3 $O/mb_$v.txt; exit 1; }
  T=$(find $O/p_$v -name "*kernel_trace.csv" | head -1)
  python tools/prof_summary.py $T --steps 21 --top 4 > $O/sum_$v.md
  echo "== $v"; sed -n 4,7p $O/sum_$v.md
done
echo KPROF_DONE
