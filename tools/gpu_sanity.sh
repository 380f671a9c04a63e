#!/bin/bash
# Session re-entry check: the GPU suite and the default bench line on the tree as built here.
#   usage: tools/gpu_sanity.sh TAG
set -o pipefail
TAG=${1:-sanity}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
echo "bench ok"
