# Where the step's time goes: phase marks on both streams (join wait), per-layer launch times
# with the D step overlapped and serialised, and a rocprofv3 kernel-trace summary of a short
# bench run.  usage: bash tools/gpu_profile.sh <outdir-name> [bench args...]
export TMPDIR=/tmp
N=${1:-profile}; shift
O=gpurun_out/$N
mkdir -p $O
bash tools/gpu_phases.sh $N/ph "$@" || exit 1
timeout -k 10 200 python tools/layer_times.py > $O/layers.txt 2>&1 || { echo "layer_times failed"; tail -5 $O/layers.txt; exit 1; }
IRGAN_NO_D_OVERLAP=1 timeout -k 10 200 python tools/layer_times.py > $O/layers_serial.txt 2>&1 || { echo "layer_times (serial) failed"; exit 1; }
head -12 $O/layers.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --kernel-steps 1 --no-cpu-baseline "$@" > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 1; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py $T --steps 8 > $O/summary.md && python tools/prof_summary.py $T --steps 8 --by-grid > $O/summary_by_grid.md
head -25 $O/summary.md
echo ALLDONE
