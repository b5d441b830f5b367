#!/bin/bash
# Like build_variant.sh, but the variant object comes from another copy of the
# source (e.g. an earlier revision): bash tools/build_variant_src.sh <name> <in-tree src> <path>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; SRC=$2; ALT=$3; shift 3
OBJDIR="$ROOT/build/native"
mkdir -p "$ROOT/variants" "$OBJDIR/variants"
INC="-I$ROOT/mpitree_amd/ops/csrc $(python -c 'import sysconfig,pybind11;print("-I"+sysconfig.get_paths()["include"],"-I"+pybind11.get_include())')"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result -D__HIP_PLATFORM_AMD__"
VOBJ="$OBJDIR/variants/$NAME.$SRC.o"
/opt/rocm/bin/hipcc $FLAGS $INC "$@" -x hip -c "$ALT" -o "$VOBJ"
OBJS=""
for o in "$OBJDIR"/*.o; do
  if [ "$(basename "$o")" = "$SRC.o" ]; then OBJS="$OBJS $VOBJ"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/variants/$NAME.so" $OBJS
echo "variants/$NAME.so"
