#!/bin/bash
# Phase-1 sweep timing at 300^3 for several round-launch grids (AIJHIP_LF_GRID).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-lfsweep}
mkdir -p "$OUT"
for g in ${GRIDS:-512 2048 8192}; do
  AIJHIP_LF_GRID=$g AIJHIP_GAMG_LOG=1 timeout -k 10 300 python -u tools/prof_case.py gamg > "$OUT/grid_$g.log" 2>&1 || exit $?
  echo "grid $g: $(grep -E 'phase 1 sweep|gamg: set-up' "$OUT/grid_$g.log" | tr '\n' ' ')"
done
