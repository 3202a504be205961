# bench.py (with CPU baseline) + rocprof kernel stats.  usage: bash tools/gpu_bench.sh <outdir-name>
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-bench}
mkdir -p $O
(nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "import os; print(len(os.sched_getaffinity(0)))") > $O/cpuinfo.txt 2>&1 || true
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
echo ALLDONE
