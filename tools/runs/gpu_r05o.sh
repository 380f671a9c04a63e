#!/bin/bash
# Round 5: the GAMG / distributed GAMG / solver GPU tests after the MIS default.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05o
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_solver_configs.py tests/test_gamg_mpi_gpu.py tests/test_gamg.py \
    tests/test_mpi_gpu.py -x -v -s -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
grep -E "ranks|its|level [0-9]:|hierarchy|CG\+GAMG" "$OUT/pytest.log" | head -40
