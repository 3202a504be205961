# serialized full GPU suite (a fault surfaces at its own test), then bench + rocprof
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r5}
mkdir -p $O
AMD_SERIALIZE_KERNEL=3 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
echo ALLDONE
