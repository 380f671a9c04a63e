#!/bin/bash
# Quick check after a kernel change: SpMV/KSP/GAMG GPU tests, then CG+Jacobi,
# CG+GAMG and the 300^3 SpMV timed, plus a kernel-stats profile of CG+GAMG.
#   usage: tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-quick}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { tail -30 "$OUT/pytest.log"; exit 1; }
for r in 1 2; do
  timeout -k 10 120 python -u tools/prof_case.py jacobi --its 400 > "$OUT/jac_$r.log" 2>&1 || exit 1
  grep 'jacobi:' "$OUT/jac_$r.log"
  timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_$r.log" 2>&1 || exit 1
  grep 'gamg: set-up' "$OUT/gamg_$r.log"
done
timeout -k 10 200 python -u tools/tune.py --variants default --rounds 5 > "$OUT/tune.jsonl" 2>&1 || exit 1
grep us_median "$OUT/tune.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 tools/prof_case.py gamg > "$OUT/prof.log" 2>&1 && echo "prof ok"
