#!/bin/bash
# Round 5: the set-up's operators (GAMG levels, P, P^T) with the gather-ordered
# copy (AIJHIP_SETUP_GSORT=1) vs without, CG + GAMG at 300^3, alternating.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ar
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gamg.py -k "gather_ordered_levels or fused_default" > "$OUT/pytest.log" 2>&1 \
  || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
for i in 1 2; do
  for g in 0 1; do
    AIJHIP_SETUP_GSORT=$g timeout -k 10 240 python -u tools/prof_case.py gamg --solves 3 > "$OUT/gamg_g${g}_$i.log" 2>&1 \
      || { tail -20 "$OUT/gamg_g${g}_$i.log"; exit 1; }
    echo "gsort $g run $i: $(grep -E '^gamg' "$OUT/gamg_g${g}_$i.log" | tr '\n' ' ')"
  done
done
