#!/bin/bash
# CG+GAMG iteration counts: the single-GPU solve of the weak-scaling grids
# (anisotropic: 300x300x600, 300x600x600) and the 300^3 operand split over 2
# and 4 ranks on one GPU (distributed GAMG vs bjacobi+GAMG), then the
# remaining GPU tests touched by this round's changes.
set -o pipefail
TAG=${1:-r03d}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
for g in "300 300 600" "300 600 600"; do
  set -- $g
  timeout -k 10 300 petsc-openacc_amd/bin/main_ksp -config configs/cg_gamg.info -da_grid_x $1 -da_grid_y $2 -da_grid_z $3 \
      > "$OUT/main_ksp_$1x$2x$3.log" 2>&1 || { tail -20 "$OUT/main_ksp_$1x$2x$3.log"; exit 1; }
  echo "single GPU $1x$2x$3:"; tail -6 "$OUT/main_ksp_$1x$2x$3.log"
done
timeout -k 10 900 python -u tools/gamg_its_ranks.py --grid 300 300 300 --ranks 2 4 > "$OUT/its_strong300.jsonl" 2> "$OUT/its_strong300.err" \
    || { tail -20 "$OUT/its_strong300.err"; exit 1; }
cat "$OUT/its_strong300.jsonl"
