# Microbench ablations of the resblock conv kernels (variant builds, tools/build_variant.sh):
# conv_pp (PP_EXP bits: 1 no MFMA, 2 no weight DMA, 4 no fragment reads, 8 no barriers, 16 no
# epilogue) on fwd+stats and dgrad; wgrad_pc (PC_EXP: 2 no DMA, 4 no fragment reads).
# usage: bash tools/gpu_ablate.sh <outdir>
export TMPDIR=/tmp
O=gpurun_out/${1:-ablate}
mkdir -p $O
B=infrared-colorization-with-resnet-generator-and-patchgan_amd/variants
for v in default pp1 pp2 pp4 pp8 pp16; do
  L=""; [ $v != default ] && L=$B/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 120 python tools/bench_conv.py --case res3x3 --which fwds,dgrad --iters 50 > $O/pp_$v.txt 2>&1 || { echo "$v failed"; break; }
  echo "$v: $(tail -1 $O/pp_$v.txt)"
done
for v in default pc2 pc4 pc6 st5 st6; do
  L=""; [ $v != default ] && L=$B/libirgan_$v.so
  IRGAN_LIB=$L timeout -k 10 120 python tools/bench_conv.py --case res3x3 --which wgrad --iters 50 > $O/pc_$v.txt 2>&1 || { echo "$v failed"; break; }
  echo "$v: $(tail -1 $O/pc_$v.txt)"
done
echo ALLDONE
