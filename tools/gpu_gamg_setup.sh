#!/bin/bash
# GAMG set-up breakdown at 300^3: per-step laps (AIJHIP_GAMG_LOG; the laps
# synchronise, so the total is a little above the bench's) of a first and a
# second set-up in one process, then rocprofv3 kernel statistics of the same
# case without the log.
#   usage: tools/gpu_gamg_setup.sh TAG
set -o pipefail
TAG=${1:-gamg_setup}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
AIJHIP_GAMG_LOG=1 timeout -k 10 300 python -u tools/prof_case.py gamg > "$OUT/setup_log.txt" 2>&1 \
  && echo "log ok" && grep -E "set-up|host phase 1|solve" "$OUT/setup_log.txt" \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
       -- python3 tools/prof_case.py gamg > "$OUT/prof_case.txt" 2>&1 && echo "prof ok" && cat "$OUT/prof_case.txt"
