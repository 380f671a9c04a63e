#!/bin/bash
# Phase-1 sweep timing at 300^3 over round-launch grids (GRIDS, AIJHIP_LF_GRID)
# and state pre-reads (PRES, AIJHIP_LF_PREREAD).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-lfsweep}
mkdir -p "$OUT"
for g in ${GRIDS:-512}; do
  for pr in ${PRES:-1}; do
    AIJHIP_LF_GRID=$g AIJHIP_LF_PREREAD=$pr AIJHIP_GAMG_LOG=1 timeout -k 10 300 python -u tools/prof_case.py gamg \
        > "$OUT/grid_${g}_pre_${pr}.log" 2>&1 || exit $?
    echo "grid $g pre $pr: $(grep -E 'phase 1 sweep rounds|staging alloc|gamg: ' "$OUT/grid_${g}_pre_${pr}.log" | tr -s ' ' | tr '\n' ' ')"
  done
done
