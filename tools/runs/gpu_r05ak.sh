#!/bin/bash
# Round 5: CG vector kernels' stores with / without the non-temporal hint
# (AIJHIP_VEC_NT=0 / 1), CG + Jacobi 400 iterations, alternating runs.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ak
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
for rep in 1 2 3; do
  for nt in 1 0; do
    AIJHIP_VEC_NT=$nt timeout -k 10 200 python -u tools/prof_case.py jacobi --its 400 > "$OUT/jac_nt${nt}_$rep.log" 2>&1 \
        || { tail -30 "$OUT/jac_nt${nt}_$rep.log"; exit 1; }
    echo "nt $nt rep $rep: $(grep -E 'jacobi:' "$OUT/jac_nt${nt}_$rep.log")"
  done
done
