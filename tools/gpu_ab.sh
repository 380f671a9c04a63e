#!/bin/bash
# A/B of two library builds in alternating processes on one box: CG+Jacobi
# (400 its), CG+GAMG solve and the default 300^3 SpMV (tools/tune.py).
#   usage: tools/gpu_ab.sh TAG LIB_A LIB_B [ROUNDS]
set -o pipefail
TAG=$1; LA=$2; LB=$3; R=${4:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
for r in $(seq 1 "$R"); do
  for side in A B; do
    lib=$LA; [[ $side == B ]] && lib=$LB
    AIJHIP_AB=1 AIJHIP_LIB=$lib timeout -k 10 120 python -u tools/prof_case.py jacobi --its 400 > "$OUT/jac_${side}_$r.log" 2>&1 || exit 1
    AIJHIP_AB=1 AIJHIP_LIB=$lib timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_${side}_$r.log" 2>&1 || exit 1
    AIJHIP_AB=1 AIJHIP_LIB=$lib timeout -k 10 200 python -u tools/tune.py --variants default --rounds 3 > "$OUT/tune_${side}_$r.jsonl" 2>&1 || exit 1
    echo "$side r$r $(grep -h 'jacobi:' "$OUT/jac_${side}_$r.log" | cut -d, -f2) | $(grep -h 'gamg: set-up' "$OUT/gamg_${side}_$r.log" | cut -d, -f2) | spmv $(grep -h '\[\\"stream' "$OUT/tune_${side}_$r.jsonl" | grep us_median | sed 's/.*us_median": \([0-9.]*\).*/\1/') us"
  done
done
