#!/bin/bash
# Round 5: the release scope of the fork / join events (tools/fence_probe.py).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05d
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/fence_probe.py --planes 38 300 --reps 100 > "$OUT/fence.jsonl" 2> "$OUT/fence.err" \
    || { tail -20 "$OUT/fence.err"; exit 1; }
cat "$OUT/fence.jsonl"
timeout -k 10 60 ./tools/bin/anyorder_probe > "$OUT/anyorder.json" 2> "$OUT/anyorder.err" \
    || { tail -20 "$OUT/anyorder.err"; exit 1; }
cat "$OUT/anyorder.json"
