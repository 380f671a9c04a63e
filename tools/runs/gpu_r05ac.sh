#!/bin/bash
# Round 5: rows over 1024 entries in blocks of their own, A/B on one box
# (AIJHIP_ISOLATE_ROW_NNZ=0 plans the old way), side stream and serial.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ac
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 400 python -u tools/ab_opts.py --case skewed --rounds 40 \
    --variant '{}' --variant '{"_env": {"AIJHIP_ISOLATE_ROW_NNZ": "0"}}' \
    --variant '{"long_overlap": 0}' --variant '{"long_overlap": 0, "_env": {"AIJHIP_ISOLATE_ROW_NNZ": "0"}}' \
    > "$OUT/ab_isolate.jsonl" 2> "$OUT/ab_isolate.err" || { tail -20 "$OUT/ab_isolate.err"; exit 1; }
cat "$OUT/ab_isolate.jsonl"
