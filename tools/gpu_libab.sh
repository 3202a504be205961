# Same-box A/B of variant builds of libirgan.so (tools/build_variant.sh): a conv
# microbench, a pytest subset and the step bench per library, interleaved.
# usage: bash tools/gpu_libab.sh <outdir> "<bench_conv.py args>" "<pytest args or ''>" <variant> [<variant> ...]
export TMPDIR=/tmp
O=gpurun_out/$1; shift
MB=$1; shift
T=$1; shift
mkdir -p $O
B=infrared-colorization-with-resnet-generator-and-patchgan_amd/variants
for v in default "$@"; do
  L=""; [ $v != default ] && L=$B/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 120 python tools/bench_conv.py $MB > $O/mb_$v.txt 2>&1 || { echo "microbench $v failed"; echo ALLDONE; exit 0; }
  echo "mb $v: $(tail -1 $O/mb_$v.txt)"
  if [ -n "$T" ]; then
    IRGAN_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > $O/t_$v.log 2>&1
    rc=$?; echo "pytest $v rc=$rc: $(tail -1 $O/t_$v.log)"
    [ $rc -ne 0 ] && { echo ALLDONE; exit 0; }
  fi
done
for rep in 1 2; do
  for v in default "$@"; do
    L=""; [ $v != default ] && L=$B/libirgan_$v.so
    IRGAN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; echo ALLDONE; exit 0; }
    python -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); print('$v', d['value'], d['ms_per_step_median'], {k.split(':')[0]: v['mean_ms'] for k, v in d['roofline']['per_kernel'].items()})"
  done
done
echo ALLDONE
