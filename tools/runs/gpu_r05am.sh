#!/bin/bash
# Round 5: the skewed stand-in's variants in the bench's order (default,
# side stream, exact, aj as stored) plus exact after the row blocks, in one
# interleaved A/B — the bench read exact (side stream) fastest.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05am
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 400 python -u tools/ab_opts.py --case skewed --rounds 40 \
    --variant '{}' --variant '{"long_overlap": 1}' --variant '{"exact": 1}' --variant '{"gather_sort": 0}' \
    --variant '{"exact": 1, "long_overlap": 0}' > "$OUT/ab.jsonl" 2> "$OUT/ab.err" || { tail -20 "$OUT/ab.err"; exit 1; }
cat "$OUT/ab.jsonl"
timeout -k 10 400 python -u tools/ab_opts.py --case skewed --rounds 40 \
    --variant '{"exact": 1}' --variant '{}' --variant '{"long_overlap": 1}' > "$OUT/ab2.jsonl" 2> "$OUT/ab2.err" \
    || { tail -20 "$OUT/ab2.err"; exit 1; }
cat "$OUT/ab2.jsonl"
