# Build an A/B variant of libirgan.so with extra -D flags on every source (tools/gpu_libab.sh,
# tools/gpu_kvar.sh): objects under build/var_<name> (not shipped), the library at
# variants/libirgan_<name>.so (shipped with the tree; load it with IRGAN_LIB=<path>).  The
# variant has the default build's source id (same sources), so _lib.load() accepts it.
# usage: bash tools/build_variant.sh <name> "-DFLAG=1 ..." ["src1.hip src2.hip": the flags on these only]
set -e
P=infrared-colorization-with-resnet-generator-and-patchgan_amd
mkdir -p $P/variants
python3 - "$1" "$2" "${3:-}" <<'PY'
import sys
sys.path.insert(0, "infrared-colorization-with-resnet-generator-and-patchgan_amd")
import _build
name, flags, only = sys.argv[1], sys.argv[2].split(), sys.argv[3].split() or None
lib = _build.build(extra_flags=flags, lib=f"{_build.HERE}/variants/libirgan_{name}.so",
                   objdir=f"{_build.OBJDIR}/var_{name}", only=only)
print(lib)
PY
