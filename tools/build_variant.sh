#!/bin/bash
# Build ablibs/<tag>/libaijhip.so from the working tree with ONE source
# file replaced by a given variant file (A/B of an edit not yet committed).
#   usage: tools/build_variant.sh TAG FILE VARIANT_PATH     (FILE relative to csrc/)
set -euo pipefail
TAG=$1; FILE=$2; SRC=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/petsc-openacc_amd/csrc
OUT=$ROOT/ablibs/$TAG
mkdir -p "$OUT"
python3 -c "import sys; sys.path.insert(0, '$ROOT'); import importlib; importlib.import_module('petsc-openacc_amd.build').build_lib()"
cp "$SRC" "$OUT/$FILE"
objs=()
for o in "$ROOT"/petsc-openacc_amd/build/*.o; do
  [[ $(basename "$o" .o) == "${FILE%.*}" ]] || objs+=("$o")
done
case $FILE in
  harness.cpp|gamg_setup.cpp) g++ -O3 -fPIC -std=c++17 -ffp-contract=off -fopenmp -I"$ROOT/include" -I"$CSRC" -c "$OUT/$FILE" -o "$OUT/${FILE%.*}.o" ;;
  *) /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wno-unused-value -I"$ROOT/include" -I"$CSRC" \
       -c "$OUT/$FILE" -o "$OUT/${FILE%.*}.o" ;;
esac
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libaijhip.so" "${objs[@]}" "$OUT/${FILE%.*}.o" \
  -lgomp -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "$OUT/libaijhip.so"
