#!/bin/bash
# Build a variant of the HIP extension with one source recompiled under extra
# -D flags (the other objects come from the last in-tree build). Output:
# variants/<name>.so, which `tools/gpu.sh ab:so=<name>` swaps in for an A/B run.
# Usage: bash tools/build_variant.sh <name> <source.hip> -DFLAG=V ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; SRC=$2; shift 2
OBJDIR="$ROOT/build/native"
mkdir -p "$ROOT/variants" "$OBJDIR/variants"
INC="-I$ROOT/mpitree_amd/ops/csrc $(python -c 'import sysconfig,pybind11;print("-I"+sysconfig.get_paths()["include"],"-I"+pybind11.get_include())')"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-result -D__HIP_PLATFORM_AMD__"
VOBJ="$OBJDIR/variants/$NAME.$SRC.o"
/opt/rocm/bin/hipcc $FLAGS $INC "$@" -c "$ROOT/mpitree_amd/ops/csrc/$SRC" -o "$VOBJ"
OBJS=""
for o in "$OBJDIR"/*.o; do
  if [ "$(basename "$o")" = "$SRC.o" ]; then OBJS="$OBJS $VOBJ"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/variants/$NAME.so" $OBJS
echo "variants/$NAME.so"
