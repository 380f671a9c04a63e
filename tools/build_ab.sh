#!/bin/bash
# Build ablibs/<tag>/libaijhip.so from the working tree with ONE source
# file taken from a git revision (default HEAD), for A/B timing of two builds
# in alternating processes: AIJHIP_LIB=ablibs/<tag>/libaijhip.so python ...
#   usage: tools/build_ab.sh TAG FILE [REV]     (FILE relative to csrc/)
set -euo pipefail
TAG=$1; FILE=$2; REV=${3:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/petsc-openacc_amd/csrc
OUT=$ROOT/ablibs/$TAG
mkdir -p "$OUT"
python3 -c "import sys; sys.path.insert(0, '$ROOT'); import importlib; importlib.import_module('petsc-openacc_amd.build').build_lib()"
git -C "$ROOT" show "$REV:petsc-openacc_amd/csrc/$FILE" > "$OUT/$FILE"
objs=()
for o in "$ROOT"/petsc-openacc_amd/build/*.o; do
  [[ $(basename "$o" .o) == "${FILE%.*}" ]] || objs+=("$o")
done
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I"$ROOT/include" -I"$CSRC" \
  -c "$OUT/$FILE" -o "$OUT/${FILE%.*}.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libaijhip.so" "${objs[@]}" "$OUT/${FILE%.*}.o" \
  -lgomp -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "$OUT/libaijhip.so"
