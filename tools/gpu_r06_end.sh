# Round-6 end evidence: smoke, bench (+CPU baseline), rocprof kernel stats of the bench, PMC
# traffic of the resblock family (bench's roofline.traffic), B=32 bf16 / fp8 and 512x640 lines.
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_end}; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 8 --warmup 3 --kernel-steps 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo rocprof failed; exit 1; }
bash tools/gpu_traffic.sh ${1:-r06_end}/traffic > $O/traffic.log 2>&1 || { echo traffic failed; exit 1; }

timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; exit 1; }
timeout -k 10 300 python bench.py --batch 32 --no-cpu-baseline > $O/bench_bf16_b32.json 2> $O/bench_bf16_b32.err || { echo b32 failed; exit 1; }
timeout -k 10 300 python bench.py --batch 32 --dtype fp8 --no-cpu-baseline > $O/bench_fp8_b32.json 2> $O/bench_fp8_b32.err || { echo fp8 failed; exit 1; }
timeout -k 10 300 python bench.py --height 512 --width 640 --batch 4 --no-cpu-baseline > $O/bench_512x640_b4.json 2> $O/bench_512.err || { echo 512 failed; exit 1; }
python - <<PY
import json
for f in ("bench", "bench_bf16_b32", "bench_fp8_b32", "bench_512x640_b4"):
    d = json.load(open("$O/%s.json" % f))
    print(f, d["value"], d["ms_per_step_median"], d["roofline"]["kernel"], d["roofline"]["frac"],
          d.get("cpu_baseline", {}).get("value"))
PY
echo ALLDONE
