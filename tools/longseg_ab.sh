#!/bin/bash
# Hub-row segment length on the skewed stand-in: one process per length
# (the planner reads AIJHIP_LONG_SEG once), default layout, 5 x 20 launches.
#   usage: tools/longseg_ab.sh TAG
set -o pipefail
TAG=${1:-longseg}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
for n in 4096 2048 8192 16384 1024; do
  AIJHIP_LONG_SEG=$n timeout -k 10 200 python -u tools/tune.py --variants geo16 --matrix skewed --rounds 3 --launches 20 \
      > "$OUT/seg_$n.jsonl" 2>&1 || { tail -5 "$OUT/seg_$n.jsonl"; exit 1; }
  echo "seg $n: $(grep '"geometry\\": 6' "$OUT/seg_$n.jsonl" | grep us_median)"
done
