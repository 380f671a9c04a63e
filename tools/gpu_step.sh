#!/bin/bash
# A short GPU call: a subset of the -m gpu suite (pytest -k EXPR), then the
# GAMG set-up breakdown (tools/gpu_gamg_setup.sh) and, optionally, one
# tools/tune.py A/B. Steps chained: the first failure ends the call.
#   usage: tools/gpu_step.sh TAG "PYTEST_K" [TUNE_ARGS...]
set -o pipefail
TAG=$1; K=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
    || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
bash tools/gpu_gamg_setup.sh "$TAG/gamg" || exit 1
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u tools/tune.py "$@" > "$OUT/tune.jsonl" 2>&1 && echo "tune ok" \
    && grep us_median "$OUT/tune.jsonl" | tail -12
fi
