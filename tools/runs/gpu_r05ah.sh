#!/bin/bash
# Round 5: the MIS set-up after the per-workgroup round counts, and the
# (r05ah: the register form of short row products).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ah
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python -u -m pytest tests/test_gamg.py tests/test_solver_configs.py tests/test_gamg_mpi_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
  for case in mis greedy; do
    if [ $case = mis ]; then opts="--gamg-opt coarsen=1 --gamg-opt eig_ksp=1"; else opts="--gamg-opt coarsen=0 --gamg-opt eig_ksp=0"; fi
    AIJHIP_GAMG_LOG=1 timeout -k 10 200 python -u tools/prof_case.py gamg $opts > "$OUT/gamg_${case}_$rep.log" 2>&1 \
        || { tail -30 "$OUT/gamg_${case}_$rep.log"; exit 1; }
    echo "$case $rep: $(grep -E 'gamg: set-up' "$OUT/gamg_${case}_$rep.log")"
  done
done
grep -E "MIS rounds|level 0 aggregate" "$OUT/gamg_mis_2.log" | head -12
grep -h "product" "$OUT/gamg_mis_2.log" | head -8
