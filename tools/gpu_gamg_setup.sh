#!/bin/bash
# GAMG set-up: the bitwise set-up tests, then the per-phase breakdown at 300^3.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-gsetup}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gamg.py \
    tests/test_solver_configs.py tests/test_ksp.py tests/test_gpu_parity.py > "$OUT/pytest.log" 2>&1 \
 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
 && AIJHIP_GAMG_LOG=1 timeout -k 10 300 python -u tools/prof_case.py gamg > "$OUT/setup.log" 2>&1 \
 && grep -E "handle|handles|phase 1|emax|strength|A\*P|P\^T|set-up|gamg:" "$OUT/setup.log" | tail -40
rc=$?; [ $rc -ne 0 ] && tail -30 "$OUT/pytest.log"; exit $rc
