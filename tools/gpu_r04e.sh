export TMPDIR=/tmp
O=gpurun_out/${1:-r04_e}
mkdir -p $O
T="python -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_step.py -k "fp32_matches or stream_overlap or bf16_close" > $O/t_step.log 2>&1 || { echo "step tests failed"; tail -5 $O/t_step.log; exit 1; }
tail -1 $O/t_step.log
timeout -k 10 300 $T tests/test_gpu_module_variants.py > $O/t_var.log 2>&1 || { echo "variant tests failed"; tail -5 $O/t_var.log; exit 1; }
tail -1 $O/t_var.log
timeout -k 10 400 $T tests/test_gpu_fp8.py > $O/t_fp8.log 2>&1
rc=$?; echo "fp8 tests rc=$rc"; tail -3 $O/t_fp8.log
[ $rc -le 1 ] && ! grep -q "+ Timeout +" $O/t_fp8.log || exit 1
bash tools/gpu_phases.sh ${1:-r04_e}/ph16 && timeout -k 10 200 python tools/layer_times.py > $O/layers.txt 2>&1 && head -60 $O/layers.txt && echo ALLDONE
