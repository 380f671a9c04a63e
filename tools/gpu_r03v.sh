#!/bin/bash
# Gather-order experiment on the skewed stand-in's ordinary rows: the same
# stream with each row block's columns sorted across the block.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-r03v}
mkdir -p "$OUT"
for mtx in skewed_nohub skewed_blocksort skewed_localx; do
  timeout -k 10 300 python3 tools/tune.py --matrix $mtx --variants geo16 --rounds 3 > "$OUT/$mtx.jsonl" 2>&1 || exit 1
  echo "== $mtx"; grep us_median "$OUT/$mtx.jsonl" | python3 -c "
import sys,json
for d in sorted((json.loads(l) for l in sys.stdin), key=lambda d: d['us_median']): print(round(d['us_median'],1), d['variant'])"
done
