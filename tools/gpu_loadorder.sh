#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-lo}
mkdir -p "$OUT"
timeout -k 10 400 python -u tools/tune.py --variants loadorder --rounds 5 > "$OUT/tune_poisson.jsonl" 2>&1 \
 && timeout -k 10 300 python -u tools/tune.py --matrix fem_hex --variants loadorder --rounds 3 > "$OUT/tune_fem.jsonl" 2>&1 \
 && timeout -k 10 300 python -u tools/tune.py --matrix skewed --variants loadorder --rounds 3 > "$OUT/tune_skewed.jsonl" 2>&1 \
 && grep -h "us_median\|bitwise" "$OUT"/tune_*.jsonl | cut -c1-160
