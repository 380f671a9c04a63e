#!/bin/bash
# Row patterns: XCD placement A/B (AIJHIP_PAT_XCHUNK) at 300^3, one process.
#   usage: tools/gpu_patxcd.sh TAG
set -o pipefail
TAG=${1:-patxcd}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/tune.py --variants patxcd --rounds 5 --launches 20 > "$OUT/tune_poisson.jsonl" 2>&1 || { tail -5 "$OUT/tune_poisson.jsonl"; exit 1; }
grep -E "us_median|bitwise" "$OUT/tune_poisson.jsonl"
