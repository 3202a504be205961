# Build an A/B variant of libirgan.so with extra -D flags on ONE source file.
# usage: bash tools/build_variant.sh <name> <source.hip> "-DFLAG=1 ..."
#   -> infrared-...amd/build/libirgan_<name>.so (load with IRGAN_LIB=<path>)
set -e
P=infrared-colorization-with-resnet-generator-and-patchgan_amd
B=$P/build
SRC=$2
OBJ=$B/var_$1_$(basename $SRC .hip).o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -I $P/csrc -Wno-unused-result $3 -c $P/csrc/$SRC -o $OBJ
OBJS=""
for s in $(python3 -c "import sys; sys.path.insert(0, '$P'); import _build; print(' '.join(x[:-4] for x in _build.SOURCES))"); do
  if [ "$s.hip" = "$SRC" ]; then OBJS="$OBJS $OBJ"; else OBJS="$OBJS $B/$s.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/libirgan_$1.so $OBJS
echo $B/libirgan_$1.so
