# round-3 parity additions + bench with the new fields.  usage: bash tools/gpu_r03a.sh <outdir>
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_bf16_elementwise.py tests/test_gpu_fused_in_bwd.py "tests/test_gpu_step.py::test_stream_overlap_schedule_bit_identical" "tests/test_gpu_step.py::test_kaist_native_resolution_512x640" "tests/test_gpu_fp8.py::test_fp8_step_vs_fp8_oracle" -s > $O/t.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
  echo "bench rc=$?"
fi
echo ALLDONE
