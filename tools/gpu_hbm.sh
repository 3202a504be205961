# HBM-bound kernel microbench (IN passes, resampling), both resample variants.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-hbm}
mkdir -p $O
timeout -k 10 120 python tools/bench_hbm.py > $O/hbm.log 2>&1
IRGAN_NO_SEP_LDS=1 timeout -k 10 120 python tools/bench_hbm.py --case up > $O/hbm_nolds.log 2>&1
IRGAN_NO_SEP_LDS=1 timeout -k 10 120 python tools/bench_hbm.py --case down >> $O/hbm_nolds.log 2>&1
echo ALLDONE
