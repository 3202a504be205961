# phase marks of the bf16 step on both streams, no profiler (IRGAN_JOIN_TIMING=1; bench.py step_phases)
export TMPDIR=/tmp
O=gpurun_out/${1:-phases}; shift
mkdir -p $O
IRGAN_JOIN_TIMING=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/bench.txt 2>&1 || { tail -5 $O/bench.txt; exit 1; }
tail -1 $O/bench.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["join_wait_ms"], d["step_phase_ms"])'
