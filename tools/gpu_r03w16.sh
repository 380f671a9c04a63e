#!/bin/bash
# 16-B LDS pair writes in the row-pattern kernel: A/B, then the GPU suite and smoke.
#   usage: tools/gpu_r03w16.sh TAG
set -o pipefail
TAG=${1:-r03w16}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu_patw16.sh "$TAG/patw16" || exit 1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || { tail -20 "$OUT/smoke.log"; exit 1; }
