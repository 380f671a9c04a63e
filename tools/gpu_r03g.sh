#!/bin/bash
# Hash-table Galerkin products + background P handles: the bitwise set-up
# tests, then set-up breakdowns at 300^3 (variants by environment).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-r03g}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gamg.py \
    tests/test_solver_configs.py tests/test_gamg_mpi_gpu.py > "$OUT/pytest.log" 2>&1 \
 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
 && AIJHIP_GAMG_LOG=1 timeout -k 10 300 python -u tools/prof_case.py gamg > "$OUT/setup_hash.log" 2>&1 \
 && AIJHIP_GAMG_AGG=device AIJHIP_GAMG_LOG=1 timeout -k 10 300 python -u tools/prof_case.py gamg > "$OUT/setup_aggdev.log" 2>&1 \
 && timeout -k 10 300 python -u tools/prof_case.py gamg > "$OUT/setup_nolog.log" 2>&1 \
 && timeout -k 10 300 python -u tools/prof_case.py gamg > "$OUT/setup_nolog2.log" 2>&1 \
 && for f in "$OUT"/setup_*.log; do echo "$(basename $f): $(grep -h 'gamg:' $f | tr '\n' ' ')"; done
rc=$?; [ $rc -ne 0 ] && tail -30 "$OUT/pytest.log"; exit $rc
