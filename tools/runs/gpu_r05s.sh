#!/bin/bash
# Round 5: non-temporal matrix loads on the headline CSR blocks and the
# stand-ins (interleaved A/B, bitwise checked).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05s
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 python -u tools/ab_opts.py --case poisson \
    --variant '{"row_patterns": 0, "column_codes": 0}' \
    --variant '{"row_patterns": 0, "column_codes": 0, "nt_loads": 1}' \
    --variant '{"row_patterns": 0, "column_codes": 0, "nt_loads": 1, "geometry": 8}' \
    --variant '{}' --variant '{"nt_loads": 1}' > "$OUT/ab_poisson.jsonl" 2> "$OUT/ab_poisson.err" \
    || { tail -20 "$OUT/ab_poisson.err"; exit 1; }
cat "$OUT/ab_poisson.jsonl"
timeout -k 10 300 python -u tools/ab_opts.py --case skewed \
    --variant '{}' --variant '{"nt_loads": 1}' --variant '{"exact": 1}' \
    > "$OUT/ab_skewed.jsonl" 2> "$OUT/ab_skewed.err" || { tail -20 "$OUT/ab_skewed.err"; exit 1; }
cat "$OUT/ab_skewed.jsonl"
timeout -k 10 300 python -u tools/ab_opts.py --case fem_hex \
    --variant '{}' --variant '{"nt_loads": 1}' > "$OUT/ab_fem.jsonl" 2> "$OUT/ab_fem.err" \
    || { tail -20 "$OUT/ab_fem.err"; exit 1; }
cat "$OUT/ab_fem.jsonl"
