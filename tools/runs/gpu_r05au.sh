#!/bin/bash
# Round 5: the gather-order sort with its last stages in registers (512
# lanes): the GPU suite, CG + GAMG at 300^3 twice, and a kernel trace of the
# set-up's sorts.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05au
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for i in 1 2; do
  timeout -k 10 240 python -u tools/prof_case.py gamg --solves 3 > "$OUT/gamg_$i.log" 2>&1 || { tail -20 "$OUT/gamg_$i.log"; exit 1; }
  echo "run $i: $(grep -E '^gamg' "$OUT/gamg_$i.log" | tr '\n' ' ')"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python3 -u tools/prof_case.py gamg > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
grep -E '^gamg' "$OUT/trace.log"
grep -h "gather_order" $(find "$OUT/prof" -name "*kernel_stats.csv") | cut -c1-200
