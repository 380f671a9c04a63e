#!/bin/bash
# Round-4 kernel probes after the record: the SpMV ladder (where the CSR
# MatMult's time goes) and the LDS x-window A/B of the CSR kernel at 300^3.
#   usage: tools/gpu_r04_probe.sh TAG
set -o pipefail
TAG=${1:-probe}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/spmv_ladder.py > "$OUT/ladder.jsonl" 2>&1 && echo "ladder ok" \
 && timeout -k 10 300 python -u tools/tune.py --variants xwin --rounds 3 > "$OUT/xwin.jsonl" 2>&1 && echo "xwin ok" \
 && grep us_median "$OUT/xwin.jsonl" && grep -v round "$OUT/ladder.jsonl" | head -3
