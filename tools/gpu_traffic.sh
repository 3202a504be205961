# HBM traffic of the resblock 3x3 conv family (fwd / dgrad / wgrad) for
# bench.py's roofline.traffic: one rocprofv3 --pmc pass per counter (FETCH_SIZE
# and WRITE_SIZE cannot share a pass), then the inference tests.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-traffic}
mkdir -p $O
for K in fwd dgrad wgrad; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$K -o run --output-format csv -- python tools/bench_conv.py --case res3x3 --iters 5 --which $K > $O/fetch_$K.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write_$K -o run --output-format csv -- python tools/bench_conv.py --case res3x3 --iters 5 --which $K > $O/write_$K.log 2>&1
done
python tools/traffic_summary.py $O > $O/traffic.json
cat $O/traffic.json

echo ALLDONE
