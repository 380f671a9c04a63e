#!/bin/bash
# Round 5: the N = 8 one-GPU rehearsal on the final tree (distributed CG +
# GAMG with the gather-ordered set-up operators, MIS across ranks).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05aw
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --gpus 8 --rehearse-one-gpu --grid 100 --strong-grid 300 --steps 20 \
    --warmup 3 > "$OUT/bench_rehearse_n8.json" 2> "$OUT/bench_rehearse_n8.err" \
    && echo "rehearsal n8 ok" || { tail -20 "$OUT/bench_rehearse_n8.err"; exit 1; }
