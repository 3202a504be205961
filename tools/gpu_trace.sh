# rocprofv3 kernel trace of a short bench run: per-kernel / per-grid summaries, per-stream gaps
# and one step's timeline per queue.  usage: bash tools/gpu_trace.sh <outdir> [extra bench args]
export TMPDIR=/tmp
O=gpurun_out/${1:-trace}; shift
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --kernel-steps 1 --no-cpu-baseline "$@" > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py $T --steps 8 > $O/summary.md && python tools/prof_summary.py $T --steps 8 --by-grid > $O/summary_by_grid.md
python tools/stream_gaps.py $T --steps 5 > $O/stream_gaps.txt
python tools/step_timeline.py $T > $O/timeline.txt
head -12 $O/summary.md; head -20 $O/stream_gaps.txt
