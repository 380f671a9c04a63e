#!/bin/bash
# GPU tuning session: parity tests first, then the interleaved variant sweep.
#   usage: tools/gpu_tune.sh TAG [tune.py args...]
set -o pipefail
TAG=${1:-tune}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > "$OUT/pytest_gpu.log" 2>&1 \
 && echo "pytest gpu ok" \
 && timeout -k 10 900 python tools/tune.py "$@" > "$OUT/tune.jsonl" 2> "$OUT/tune.err" \
 && echo "tune ok"
rc=$?
tail -3 "$OUT/pytest_gpu.log"
tail -30 "$OUT/tune.jsonl" 2>/dev/null
exit $rc
