#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-nt}
mkdir -p "$OUT"
timeout -k 10 120 tools/read_sweep > "$OUT/sweep.jsonl" 2>&1 \
 && timeout -k 10 400 python -u tools/tune.py --variants ntgeom --rounds 4 > "$OUT/tune_poisson.jsonl" 2>&1 \
 && timeout -k 10 300 python -u tools/tune.py --matrix fem_hex --variants ntgeom --rounds 3 > "$OUT/tune_fem.jsonl" 2>&1 \
 && cat "$OUT/sweep.jsonl" && grep us_median "$OUT"/tune_*.jsonl
