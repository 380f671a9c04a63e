#!/bin/bash
# After the block-relative column layout: its tests first, then the whole
# -m gpu suite, then CG + GAMG timed (layout on / off on the levels through
# the fine handle's column_codes) and the set-up breakdown. Chained.
set -o pipefail
TAG=${1:-s7}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_column_codes_gpu.py -x -v --timeout 200 --timeout-method thread \
    > "$OUT/pytest_codes.log" 2>&1 && tail -1 "$OUT/pytest_codes.log" || { grep -E "FAIL|Error|assert" "$OUT/pytest_codes.log" | tail -20; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    && tail -1 "$OUT/pytest.log" || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
for r in 1 2; do
  timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_rel_$r.log" 2>&1 || exit 1
done
grep -H "set-up" "$OUT"/gamg_rel_*.log
bash tools/gpu_gamg_setup.sh "$TAG/gamg" | tail -3
