#!/bin/bash
# Round 5: the parity file with the new planner / overlap tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ai
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && tail -1 "$OUT/pytest.log" || { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
grep -E "isolate|own_block|overlap_auto" "$OUT/pytest.log"
