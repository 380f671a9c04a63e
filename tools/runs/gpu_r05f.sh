#!/bin/bash
# Round 5: the fork / join decomposed (tools/halo_probe.py), at 4 and 8
# hardware queues.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05f
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
for q in 8 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/halo_probe.py --grid 300 --planes 38 300 --reps 200 \
      --only diag,forkjoin,rec_only,fork_only,join_done,join_fresh,ag_empty,p2p_empty,p2p_selfd,p2p_self,ag_self \
      > "$OUT/halo_q$q.jsonl" 2> "$OUT/halo_q$q.err" || { tail -20 "$OUT/halo_q$q.err"; exit 1; }
  cat "$OUT/halo_q$q.jsonl"
done
