# Round-6 pass l: rocprofv3 kernel stats of the config-5 (fp8, B=32) and config-4 shape
# (512x640, B=4) bench lines
export TMPDIR=/tmp
O=gpurun_out/r06_l; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fp8 -o run --output-format csv -- python bench.py --batch 32 --dtype fp8 --steps 8 --warmup 3 --kernel-steps 2 --no-cpu-baseline > $O/bench_fp8.json 2> $O/prof_fp8.log || { echo prof fp8 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_512 -o run --output-format csv -- python bench.py --height 512 --width 640 --batch 4 --steps 8 --warmup 3 --kernel-steps 2 --no-cpu-baseline > $O/bench_512.json 2> $O/prof_512.log || { echo prof 512 failed; exit 1; }
ls $O/prof_fp8 $O/prof_512
echo ALLDONE
