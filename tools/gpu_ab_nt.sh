#!/bin/bash
# DIAGNOSTIC: GPU suite, then the non-temporal-store A/B (tools/ab_vec_nt.py), then a bench line.
set -o pipefail
TAG=${1:-abnt}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -x -q -m gpu > "$OUT/pytest_gpu.log" 2>&1 \
 && echo "pytest gpu ok" \
 && timeout -k 10 300 python3 tools/ab_vec_nt.py > "$OUT/ab_vec_nt.jsonl" 2> "$OUT/ab_vec_nt.err" \
 && echo "ab ok" && cat "$OUT/ab_vec_nt.jsonl" \
 && timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" \
 && echo "bench ok" && cat "$OUT/bench.json"
rc=$?
tail -3 "$OUT/pytest_gpu.log"
exit $rc
