# conv microbench of every training shape (tools/bench_conv.py) under a rocprofv3 kernel trace:
# isolated per-case times and which kernel each case launches (tools/case_kernels.py)
export TMPDIR=/tmp
O=gpurun_out/${1:-convcases}; shift
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python tools/bench_conv.py --iters 10 "$@" > $O/bench.txt 2>&1 || { tail -5 $O/bench.txt; exit 1; }
K=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/case_kernels.py $K --iters 10 > $O/case_kernels.txt && cat $O/case_kernels.txt && grep "ms/TFLOPs" $O/bench.txt
