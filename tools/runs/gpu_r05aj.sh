#!/bin/bash
# Round 5: the V-cycle's plain-block kernels (coarse levels, P, P^T) on the
# branch-free phase 1 (AIJHIP_PLAIN_BF=1) vs predicated, alternating runs.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05aj
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
for rep in 1 2 3; do
  for bf in 0 1; do
    AIJHIP_PLAIN_BF=$bf timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_bf${bf}_$rep.log" 2>&1 \
        || { tail -30 "$OUT/gamg_bf${bf}_$rep.log"; exit 1; }
    echo "bf $bf rep $rep: $(grep -E 'gamg: set-up' "$OUT/gamg_bf${bf}_$rep.log")"
  done
done
