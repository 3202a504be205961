# Kernel trace + HIP runtime trace of a short bench run (no counters), and the host-enqueue
# vs GPU-start table of one step (tools/launch_lag.py).  usage: bash tools/gpu_apitrace.sh <outdir> [bench args]
export TMPDIR=/tmp
O=gpurun_out/${1:-apitrace}; shift
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --kernel-steps 1 --no-cpu-baseline "$@" > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
K=$(find $O/prof -name "*kernel_trace.csv" | head -1)
A=$(find $O/prof -name "*hip_api_trace.csv" | head -1)
python tools/launch_lag.py $K $A > $O/launch_lag.txt && python tools/step_timeline.py $K > $O/timeline.txt
head -3 $O/launch_lag.txt; tail -25 $O/launch_lag.txt
