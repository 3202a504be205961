set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/p2
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -k conv > gpurun_out/p2/pytest_conv.log 2>&1
timeout -k 10 200 python tools/bench_conv.py --iters 20 > gpurun_out/p2/bench_halo.log 2>&1
IRGAN_NO_HALO=1 timeout -k 10 200 python tools/bench_conv.py --iters 20 > gpurun_out/p2/bench_nohalo.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d gpurun_out/p2/pmc_sq -o run --output-format csv -- python tools/bench_conv.py --case res3x3 --which fwd --iters 5 > gpurun_out/p2/pmc_sq.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d gpurun_out/p2/pmc_tcc -o run --output-format csv -- python tools/bench_conv.py --case res3x3 --which fwd --iters 5 > gpurun_out/p2/pmc_tcc.log 2>&1
echo ALLDONE
