# Bench A/B: the default build against env switches, no CPU baseline.
# usage: bash tools/gpu_bench_ab.sh <outdir-name> <ENV=VALUE> [<ENV=VALUE> ...]
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}
shift
mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_base.json 2> $O/bench_base.err
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err
  echo "$i $e" >> $O/variants.txt
done
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_base2.json 2> $O/bench_base2.err
echo ALLDONE
