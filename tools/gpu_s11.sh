#!/bin/bash
# The fused CG p-update: the KSP / solver tests first, the whole -m gpu
# suite, then CG + Jacobi and CG + GAMG timed fused vs separate (in turn).
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/s11
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ksp.py tests/test_solver_configs.py tests/test_row_patterns_gpu.py -x -q -m gpu \
    --timeout 200 --timeout-method thread > "$OUT/pytest_ksp.log" 2>&1 && tail -1 "$OUT/pytest_ksp.log" \
    || { grep -E "FAIL|Error|assert" "$OUT/pytest_ksp.log" | tail -20; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    && tail -1 "$OUT/pytest.log" || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
for r in 1 2 3; do
  timeout -k 10 120 python -u tools/prof_case.py jacobi --its 400 > "$OUT/jac_fused_$r.log" 2>&1 || exit 1
  AIJHIP_CG_PSEP=1 timeout -k 10 120 python -u tools/prof_case.py jacobi --its 400 > "$OUT/jac_sep_$r.log" 2>&1 || exit 1
  timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_fused_$r.log" 2>&1 || exit 1
  AIJHIP_CG_PSEP=1 timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_sep_$r.log" 2>&1 || exit 1
done
grep -H "jacobi:\|gamg: set-up" "$OUT"/jac_*.log "$OUT"/gamg_*.log
