set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-abl}
mkdir -p $O
for m in 0 1 2 3 4 7 0; do
  IRGAN_PP_DBG=$m timeout -k 10 100 python tools/bench_conv.py --iters 50 --case res3 --which fwd >> $O/abl.log 2>&1
  echo "mode $m done" >> $O/abl.log
done
echo ALLDONE
