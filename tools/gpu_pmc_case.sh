#!/bin/bash
# Kernel trace + HBM-traffic PMC passes of one tools/prof_case.py workload
# (one rocprofv3 pass per counter group; --pmc only with kernel tracing).
#   usage: tools/gpu_pmc_case.sh TAG CASE [prof_case args...]
set -o pipefail
TAG=${1:-pmccase}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/prof_case.py $CASE \
    > "$OUT/$name.log" 2>&1
}
CASE="$*"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 tools/prof_case.py $CASE > "$OUT/trace.log" 2>&1 \
 && run fetch FETCH_SIZE \
 && run write WRITE_SIZE \
 && run tcc TCC_HIT_sum TCC_MISS_sum \
 && run ea TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
 && run grbm GRBM_GUI_ACTIVE GRBM_COUNT \
 && python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
