# Round-6 pass w: head kernels alone under rocprofv3 (dedicated vs generic), then the tests
export TMPDIR=/tmp
O=gpurun_out/r06_w; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_head -o run --output-format csv -- python3 tools/head_prof.py > $O/prof_head.log 2>&1 || { echo prof failed; tail $O/prof_head.log; exit 1; }
IRGAN_HEAD_FWD_SPLIT=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_gen -o run --output-format csv -- python3 tools/head_prof.py > $O/prof_gen.log 2>&1 || { echo prof2 failed; exit 1; }
python tools/kernel_trace_summary.py $O/prof_head/run_kernel_trace.csv $O/prof_gen/run_kernel_trace.csv
timeout -k 10 300 python -u -m pytest tests/test_gpu_patch_head.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$? $(tail -1 $O/pytest.log)"
