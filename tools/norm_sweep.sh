# IN pass microbenchmark under environment switches.  usage: bash tools/norm_sweep.sh <outdir> "<ENV=1 ...>" ...
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 200 python tools/norm_bench.py > $O/nb_default.txt 2>&1 || { echo "norm_bench failed"; exit 1; }
for envs in "$@"; do
  tag=$(echo $envs | tr ' =' '__')
  timeout -k 10 200 env $envs python tools/norm_bench.py > $O/nb_$tag.txt 2>&1 || { echo "norm_bench $envs failed"; exit 1; }
done
grep -H "" $O/nb_*.txt | grep "N=16"
