# Same-box A/B of InstanceNorm pass variants (tools/build_variant.sh): tools/norm_bench.py and
# the step bench per library, interleaved.  usage: bash tools/gpu_normab.sh <outdir> <variant> ...
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
B=infrared-colorization-with-resnet-generator-and-patchgan_amd/variants
for v in default "$@"; do
  L=""; [ $v != default ] && L=$B/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 120 python tools/norm_bench.py > $O/nb_$v.txt 2>&1 || { echo "norm bench $v failed"; tail -3 $O/nb_$v.txt; exit 1; }
  echo "== $v"; cat $O/nb_$v.txt | grep -v amdgpu.ids
done
for rep in 1 2; do
  for v in default "$@"; do
    L=""; [ $v != default ] && L=$B/libirgan_$v.so
    IRGAN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); print('$v', d['value'], d['ms_per_step_median'], {k.split(':')[0]: v['mean_ms'] for k, v in d['roofline']['hbm_kernels'].items()})"
  done
done
echo ALLDONE
