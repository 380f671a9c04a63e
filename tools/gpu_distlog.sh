#!/bin/bash
# The distributed GAMG set-up's per-step log at world size 1 (forced), 300^3.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-distlog}
mkdir -p "$OUT"
AIJHIP_GAMG_DIST=1 AIJHIP_GAMG_LOG=1 timeout -k 10 300 python3 tools/gamg_its_ranks.py --grid 300 300 300 --ranks 1 \
    --pcs gamg > "$OUT/dist1.log" 2>&1; rc=$?; tail -3 "$OUT/dist1.log"; exit $rc
