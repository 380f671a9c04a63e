#!/bin/bash
# DIAGNOSTIC: STREAM block-shape / load-form study on the GPU box.
set -o pipefail
TAG=${1:-abuf}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/ablate_buf.py > "$OUT/ablate_buf.jsonl" 2> "$OUT/ablate_buf.err" \
 && echo "ablate ok" && cat "$OUT/ablate_buf.jsonl"
