#!/bin/bash
# The skewed Flan_1565 stand-in: the long-row launch forms A/B'd in one
# process, then per-kernel statistics and a kernel trace of the default plan
# and of the side-stream form (which launches run concurrently).
#   usage: tools/gpu_skewed.sh TAG
set -o pipefail
TAG=${1:-skewed}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/tune.py --matrix skewed --variants overlap --rounds 5 > "$OUT/overlap.jsonl" 2>&1 \
    && echo "overlap ok" && grep us_median "$OUT/overlap.jsonl" | tail -6 || exit 1
for ov in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_ov$ov" -o run --output-format csv \
      -- python3 tools/prof_case.py skewed --its 50 --opt long_overlap=$ov > "$OUT/prof_ov$ov.log" 2>&1 \
      && echo "prof ov$ov ok" && python3 tools/trace_gaps.py "$OUT/prof_ov$ov" --last 300 | head -12 || exit 1
done
