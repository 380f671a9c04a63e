#!/bin/bash
# Round 5: block geometries with fewer pairs per lane on the headline CSR
# blocks (the flat read's fastest shape is two 16-B loads per lane).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05t
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 python -u tools/ab_opts.py --case poisson \
    --variant '{"row_patterns": 0, "column_codes": 0}' \
    --variant '{"row_patterns": 0, "column_codes": 0, "geometry": 9}' \
    --variant '{"row_patterns": 0, "column_codes": 0, "geometry": 5}' \
    --variant '{"row_patterns": 0, "column_codes": 0, "geometry": 0}' \
    --variant '{"row_patterns": 0, "column_codes": 0, "geometry": 1}' > "$OUT/ab_geom.jsonl" 2> "$OUT/ab_geom.err" \
    || { tail -20 "$OUT/ab_geom.err"; exit 1; }
cat "$OUT/ab_geom.jsonl"
