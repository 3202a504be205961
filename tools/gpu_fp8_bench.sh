# Config-5 bench lines (256x256, B=32): fp8 and bf16 side by side, plus rocprof
# kernel stats of the fp8 run.  usage: bash tools/gpu_fp8_bench.sh <outdir-name>
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-fp8bench}
mkdir -p $O
timeout -k 10 300 python bench.py --batch 32 --dtype fp8 --steps 20 --no-cpu-baseline > $O/bench_fp8.json 2> $O/bench_fp8.err
timeout -k 10 300 python bench.py --batch 32 --dtype bf16 --steps 20 --no-cpu-baseline > $O/bench_bf16_b32.json 2> $O/bench_bf16_b32.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --batch 32 --dtype fp8 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
echo ALLDONE
