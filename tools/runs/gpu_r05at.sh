#!/bin/bash
# Round 5: the set-up's long-row operators gather-ordered by default (32-bit
# columns where the 16-bit form does not fit): the GPU suite, then CG + GAMG
# at 300^3 default / off (0) / every operator (1), alternating.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05at
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for i in 1 2; do
  for g in def 0 1; do
    if [ $g = def ]; then unset AIJHIP_SETUP_GSORT; else export AIJHIP_SETUP_GSORT=$g; fi
    timeout -k 10 240 python -u tools/prof_case.py gamg --solves 3 > "$OUT/gamg_${g}_$i.log" 2>&1 \
      || { tail -20 "$OUT/gamg_${g}_$i.log"; exit 1; }
    echo "gsort $g run $i: $(grep -E '^gamg' "$OUT/gamg_${g}_$i.log" | tr '\n' ' ')"
  done
done
