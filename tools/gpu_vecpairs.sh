#!/bin/bash
# CG vector kernels over element pairs: KSP tests, then A/B of
# AIJHIP_VEC_PAIRS=1/0 on CG+Jacobi (200 its) and CG+GAMG at 300^3.
#   usage: tools/gpu_vecpairs.sh TAG
set -o pipefail
TAG=${1:-vp}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ksp.py tests/test_ksp_mpi.py tests/test_gamg.py -x -q -m gpu \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 && echo "pytest ok" || { tail -30 "$OUT/pytest.log"; exit 1; }
for r in 1 2; do
  for vp in 1 0; do
    AIJHIP_VEC_PAIRS=$vp timeout -k 10 120 python -u tools/prof_case.py jacobi --its 400 > "$OUT/jac_${vp}_$r.log" 2>&1 || exit 1
    echo "pairs=$vp $(grep 'jacobi:' "$OUT/jac_${vp}_$r.log")"
  done
done
for vp in 1 0; do
  AIJHIP_VEC_PAIRS=$vp timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_$vp.log" 2>&1 || exit 1
  echo "pairs=$vp $(grep 'gamg: set-up' "$OUT/gamg_$vp.log")"
done
