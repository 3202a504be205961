# round-4: last-block IN finalize + fp8 reflect-line dgrad (tests), contention study (phases and
# per-layer times with the D step overlapped vs serialised), W2 ablations
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_f}
mkdir -p $O
T="python -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_bf16_elementwise.py tests/test_gpu_kernels.py > $O/t_el.log 2>&1 || { echo "elementwise tests failed"; tail -8 $O/t_el.log; exit 1; }
tail -1 $O/t_el.log
timeout -k 10 400 $T tests/test_gpu_fp8.py tests/test_gpu_ring_epi.py > $O/t_fp8.log 2>&1 || { echo "fp8 tests failed"; tail -8 $O/t_fp8.log; exit 1; }
tail -1 $O/t_fp8.log
timeout -k 10 300 $T tests/test_gpu_step.py -k "fp32_matches or stream_overlap or bf16_close" > $O/t_step.log 2>&1 || { echo "step tests failed"; tail -5 $O/t_step.log; exit 1; }
tail -1 $O/t_step.log
bash tools/gpu_phases.sh ${1:-r04_f}/ph || exit 1
IRGAN_NO_VGG_OVERLAP=1 bash tools/gpu_phases.sh ${1:-r04_f}/ph_novgg || exit 1
IRGAN_NO_D_OVERLAP=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/serial.txt 2>&1 || exit 1
echo "serial: $(tail -1 $O/serial.txt | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
IRGAN_NO_D_OVERLAP=1 timeout -k 10 200 python tools/layer_times.py > $O/layers_serial.txt 2>&1 || exit 1
bash tools/gpu_kvar.sh ${1:-r04_f}/w2 "--case res3x3 --which wgrad --iters 20" w2x1 w2x2 w2x4 w2x8
