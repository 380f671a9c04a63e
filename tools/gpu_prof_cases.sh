#!/bin/bash
# Kernel breakdowns of the CG+GAMG solve, CG+Jacobi and the skewed SpMV
# (rocprofv3 --kernel-trace --stats, one process per case, own time limits).
#   usage: tools/gpu_prof_cases.sh TAG
set -o pipefail
TAG=${1:-cases}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
AIJHIP_GAMG_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/gamg" -o run --output-format csv \
    -- python3 tools/prof_case.py gamg > "$OUT/gamg.log" 2>&1 \
 && echo "gamg ok" && grep -v "^gamg level [2-9]" "$OUT/gamg.log" | tail -25 \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/skewed" -o run --output-format csv \
    -- python3 tools/prof_case.py skewed > "$OUT/skewed.log" 2>&1 \
 && echo "skewed ok"
