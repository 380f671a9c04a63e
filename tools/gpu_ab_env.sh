#!/bin/bash
# A/B of one environment switch in alternating processes: CG+Jacobi (400
# its) and CG+GAMG solve via tools/prof_case.py.
#   usage: tools/gpu_ab_env.sh TAG VAR VALUE_A VALUE_B ROUNDS
set -o pipefail
TAG=$1; VAR=$2; VA=$3; VB=$4; R=${5:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
for r in $(seq 1 "$R"); do
  for side in A B; do
    v=$VA; [[ $side == B ]] && v=$VB
    env "$VAR=$v" timeout -k 10 120 python -u tools/prof_case.py jacobi --its 400 > "$OUT/jac_${side}_$r.log" 2>&1 || exit 1
    env "$VAR=$v" timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_${side}_$r.log" 2>&1 || exit 1
    echo "$side ($VAR=$v) r$r $(grep -h 'jacobi:' "$OUT/jac_${side}_$r.log" | cut -d, -f2) | $(grep -h 'gamg: set-up' "$OUT/gamg_${side}_$r.log" | cut -d, -f1,2)"
  done
done
