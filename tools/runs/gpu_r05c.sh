#!/bin/bash
# Round 5: the halo probe without graphs (device-only and pipelined costs of
# the fork / join, the deferred RCCL collective), then — last, since it
# crashed the probe in r05b — the HIP-graph capture of the diagonal block
# alone under faulthandler, to find where.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05c
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/halo_probe.py --grid 300 --planes 300 38 --reps 200 --graphs 0 > "$OUT/halo.jsonl" \
    2> "$OUT/halo.err" || { tail -20 "$OUT/halo.err"; exit 1; }
cat "$OUT/halo.jsonl"
timeout -k 10 120 python -X faulthandler -u tools/halo_probe.py --grid 300 --planes 38 --reps 20 --burst 20 \
    --only diag,diag_graph > "$OUT/graph_diag.jsonl" 2> "$OUT/graph_diag.err"
echo "graph diag rc=$?"
tail -40 "$OUT/graph_diag.err"
cat "$OUT/graph_diag.jsonl"
