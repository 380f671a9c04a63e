#!/bin/bash
# Round 5: the fork / join release scope, one mode per process, at HIP's
# default 4 hardware queues and at 8, interleaved twice.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05e
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
for rep in 1 2; do
  for q in 4 8; do
    for f in system device; do
      GPU_MAX_HW_QUEUES=$q AIJHIP_EVENT_FENCE=$f timeout -k 10 200 python -u tools/fence_probe.py --per-process \
          --planes 38 --reps 100 >> "$OUT/fence_pp.jsonl" 2>> "$OUT/fence_pp.err" \
          || { tail -20 "$OUT/fence_pp.err"; exit 1; }
    done
  done
done
cat "$OUT/fence_pp.jsonl"
