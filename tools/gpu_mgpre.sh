#!/bin/bash
# V-cycle pre-smoothing A/B: AIJHIP_MG_PRE_SPLIT=0 (one launch, two gathers)
# vs 1 (x = D^-1 b pass + residual SpMV), CG+GAMG at 300^3, interleaved.
#   usage: tools/gpu_mgpre.sh TAG
set -o pipefail
TAG=${1:-mgpre}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
for r in 1 2; do
  for sp in 1 0; do
    AIJHIP_MG_PRE_SPLIT=$sp timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_${sp}_$r.log" 2>&1 || exit 1
    echo "split=$sp $(grep 'gamg: set-up' "$OUT/gamg_${sp}_$r.log")"
  done
done
AIJHIP_MG_PRE_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 tools/prof_case.py gamg > "$OUT/prof.log" 2>&1 && echo "prof ok"
