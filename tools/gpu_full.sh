#!/bin/bash
# Full GPU check: every -m gpu test, then the default bench line.
#   usage: tools/gpu_full.sh TAG [bench args...]
set -o pipefail
TAG=${1:-full}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 \
 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
 && timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
 && echo "bench ok" && cat "$OUT/bench.json"
rc=$?
[ $rc -ne 0 ] && tail -40 "$OUT/pytest.log" && tail -20 "$OUT/bench.err" 2>/dev/null
exit $rc
