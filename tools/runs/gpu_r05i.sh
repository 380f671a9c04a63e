#!/bin/bash
# Round 5: the MIS set-up after the emax stream / first-round / device-rule
# changes: GAMG GPU tests, then the set-up logs of both hierarchies.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05i
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python -u -m pytest tests/test_gamg.py tests/test_solver_configs.py tests/test_ksp.py -x -v -m gpu \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for case in mis greedy; do
  if [ $case = mis ]; then opts="--gamg-opt coarsen=1 --gamg-opt eig_ksp=1"; else opts=""; fi
  AIJHIP_GAMG_LOG=1 timeout -k 10 200 python -u tools/prof_case.py gamg $opts > "$OUT/gamg_$case.log" 2>&1 \
      || { tail -30 "$OUT/gamg_$case.log"; exit 1; }
  grep -E "gamg:" "$OUT/gamg_$case.log"
done
