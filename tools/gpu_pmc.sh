#!/bin/bash
# HBM-traffic counters for the SpMV kernel, one rocprofv3 pass per counter
# group (MI355X_MICROARCH.md §rocprofv3 PMC slots: FETCH_SIZE and WRITE_SIZE
# do not fit one pass). --pmc only with kernel tracing; no sys/runtime trace.
#   usage: tools/gpu_pmc.sh TAG [bench args...]
set -o pipefail
TAG=${1:-pmc}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
B="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cg --no-gamg $*"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 $B \
    > "$OUT/$name.log" 2>&1
}
timeout -k 10 300 python3 $B > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $B \
      > "$OUT/trace.log" 2>&1 \
 && run fetch FETCH_SIZE \
 && run write WRITE_SIZE \
 && run tcc TCC_HIT_sum TCC_MISS_sum \
 && run ea TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
 && run grbm GRBM_GUI_ACTIVE GRBM_COUNT \
 && python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
