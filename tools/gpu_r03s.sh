#!/bin/bash
# The distributed GAMG set-up after its host round trips went to the device:
# the multi-rank GPU tests, then the per-step log at world size 1 (forced).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-r03s}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gamg_mpi_gpu.py \
    tests/test_mpi_gpu.py tests/test_comm_gpu.py > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
 && AIJHIP_GAMG_DIST=1 AIJHIP_GAMG_LOG=1 timeout -k 10 300 python3 tools/gamg_its_ranks.py --grid 300 300 300 --ranks 1 \
    --pcs gamg > "$OUT/dist1.log" 2>&1 && grep -E "gamg mpi level [01]|\"its\"" "$OUT/dist1.log" | tail -30
rc=$?; [ $rc -ne 0 ] && tail -30 "$OUT/pytest.log"; exit $rc
