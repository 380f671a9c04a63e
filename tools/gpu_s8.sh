#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/s8
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/tune.py --matrix banded --variants rel --rounds 5 > "$OUT/rel_banded.jsonl" 2>&1 \
  && grep -h "bitwise\|us_median" "$OUT/rel_banded.jsonl" | cut -c1-200 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_rel_$r.log" 2>&1 || exit 1
  AIJHIP_GAMG_REL0=1 timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_aj_$r.log" 2>&1 || exit 1
done
grep -H "gamg: set-up" "$OUT"/gamg_*.log
