#!/bin/bash
# One GPU-box session: smoke, parity tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the session (no retries).
#   usage: tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
echo "== rocm-smi" && (rocm-smi --showproductname > "$OUT/smi.txt" 2>&1 || true)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
 && echo "smoke ok" \
 && timeout -k 10 900 python -m pytest tests -x -q -m gpu > "$OUT/pytest_gpu.log" 2>&1 \
 && echo "pytest gpu ok" \
 && timeout -k 10 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
 && echo "bench ok" && cat "$OUT/bench.json" \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
      -- python3 bench.py --steps 100 --no-cpu-baseline --no-cg --no-gamg --no-host-vec "$@" > "$OUT/prof.log" 2>&1 \
 && echo "rocprof ok"
rc=$?
tail -5 "$OUT/pytest_gpu.log" 2>/dev/null
exit $rc
