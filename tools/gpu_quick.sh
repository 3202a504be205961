# one test file + bench (no CPU baseline).  usage: bash tools/gpu_quick.sh <outdir> <test file>
set -e
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest $2 -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], {k:v['mean_ms'] for k,v in d['roofline']['per_kernel'].items()})"
echo ALLDONE
