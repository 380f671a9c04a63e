#!/bin/bash
# SQ wait / issue counters (one rocprofv3 --pmc pass per case, kernel trace
# beside them) of tools/prof_case.py cases: default layout and kernel.
#   usage: tools/pmc_sq.sh TAG CASE...      (e.g. skewed poisson)
set -o pipefail
TAG=${1:-sq}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES"
for case in "$@"; do
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -d "$OUT/$case" -o run --output-format csv \
    -- python3 tools/prof_case.py $case --its 10 > "$OUT/$case.log" 2>&1 || exit 1
  echo "sq $case ok"
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary_all.json" 2>/dev/null; tail -c 1500 "$OUT/summary_all.json"
