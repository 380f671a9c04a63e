#!/bin/bash
# Round 5: where PETSc's MIS coarsening's set-up goes (AIJHIP_GAMG_LOG) beside
# the greedy one, then the eight-rank one-GPU rehearsal with progress lines.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05h
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
AIJHIP_GAMG_LOG=1 timeout -k 10 200 python -u tools/prof_case.py gamg --gamg-opt coarsen=1 --gamg-opt eig_ksp=1 \
    > "$OUT/gamg_mis.log" 2>&1 || { tail -30 "$OUT/gamg_mis.log"; exit 1; }
grep -E "gamg:|MIS|emax|level 0|level 1" "$OUT/gamg_mis.log" | head -60
AIJHIP_GAMG_LOG=1 timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_greedy.log" 2>&1 \
    || { tail -30 "$OUT/gamg_greedy.log"; exit 1; }
grep -E "gamg:" "$OUT/gamg_greedy.log"
timeout -k 10 900 python -u bench.py --gpus 8 --rehearse-one-gpu --grid 60 --strong-grid 300 --steps 20 \
    --warmup 3 > "$OUT/bench_rehearse_n8.json" 2> "$OUT/bench_rehearse_n8.err" \
    && echo "rehearsal n8 ok" || { tail -30 "$OUT/bench_rehearse_n8.err"; exit 1; }
