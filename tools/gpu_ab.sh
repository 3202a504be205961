# Tests, then a same-box bench A/B of environment switches.
# usage: bash tools/gpu_ab.sh <outdir> "<pytest targets>" "<ENV=1 ...>" ["<ENV=1 ...>" ...]
#   each switch set runs bench.py twice, interleaved with the default, no CPU baseline
export TMPDIR=/tmp
O=gpurun_out/$1; shift
T=$1; shift
mkdir -p $O
if [ -n "$T" ]; then
  timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread $T > $O/t.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/t.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo ALLDONE; exit 0; fi
fi
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default_$rep.json 2> $O/bench_default_$rep.err || { echo "bench default failed"; break; }
  python -c "import json; d=json.load(open('$O/bench_default_$rep.json')); print('default', d['value'], {k.split(':')[0]: v['mean_ms'] for k, v in d['roofline']['per_kernel'].items()})"
  for envs in "$@"; do
    tag=$(echo $envs | tr ' =' '__')
    timeout -k 10 300 env $envs python bench.py --no-cpu-baseline > $O/bench_${tag}_$rep.json 2> $O/bench_${tag}_$rep.err || { echo "bench $envs failed"; break 2; }
    python -c "import json; d=json.load(open('$O/bench_${tag}_$rep.json')); print('$envs', d['value'], {k.split(':')[0]: v['mean_ms'] for k, v in d['roofline']['per_kernel'].items()})"
  done
done
echo ALLDONE
