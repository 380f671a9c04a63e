#!/bin/bash
# Round 5: the skewed stand-in without its hub rows (what the row blocks
# alone reach), layouts A/B; the flat read for scale comes from the bench.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05w
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 python -u tools/ab_opts.py --case skewed_nohub \
    --variant '{}' --variant '{"gather_sort": 0}' --variant '{"gather_sort": 0, "column_codes": 1}' \
    --variant '{"exact": 1}' > "$OUT/ab_nohub.jsonl" 2> "$OUT/ab_nohub.err" || { tail -20 "$OUT/ab_nohub.err"; exit 1; }
cat "$OUT/ab_nohub.jsonl"
timeout -k 10 300 python -u tools/ab_opts.py --case skewed \
    --variant '{}' --variant '{"long_overlap": 0}' --variant '{"long_xcd": 0}' \
    > "$OUT/ab_skewed.jsonl" 2> "$OUT/ab_skewed.err" || { tail -20 "$OUT/ab_skewed.err"; exit 1; }
cat "$OUT/ab_skewed.jsonl"
grep -h "ab_opts: {}" "$OUT"/*.err | cut -c1-600
