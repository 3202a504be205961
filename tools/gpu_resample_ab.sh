set -e
export TMPDIR=/tmp
for r in 1 2; do for E in IRGAN_SEP_SWZ=0 IRGAN_SEP_SWZ=1; do echo "## $E"; env $E timeout -k 10 100 python tools/resample_bench.py; done; done
