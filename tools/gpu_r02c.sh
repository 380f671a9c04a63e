#!/bin/bash
# r02c: full bench (same-run read ceiling) + its kernel stats, then PMC of
# the skewed stand-in and of the 300^3 SpMV with the plane-chunk XCD remap.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r02c
mkdir -p "$OUT"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && echo "bench ok" \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
      -- python3 bench.py --steps 100 --no-cpu-baseline --no-cg --no-gamg --no-host-vec > "$OUT/prof.log" 2>&1 \
 && echo "prof ok" \
 && tools/gpu_pmc_case.sh r02c_pmc_skewed skewed --its 30 > /dev/null && echo "pmc skewed ok" \
 && tools/gpu_pmc_case.sh r02c_pmc_xchunk22 poisson --its 30 --opt xcd_remap=22 > /dev/null && echo "pmc xchunk ok" \
 && tools/gpu_pmc_case.sh r02c_pmc_default poisson --its 30 > /dev/null && echo "pmc default ok"
