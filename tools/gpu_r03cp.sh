#!/bin/bash
# Profiles of the coded headline: rocprofv3 kernel statistics of the bench's
# headline alone, then the HBM-traffic PMC passes of 300^3 SpMVs with the
# automatic layout (column codes) and with aj (column_codes=0).
#   usage: tools/gpu_r03cp.sh TAG
set -o pipefail
TAG=${1:-r03cp}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_headline" -o run --output-format csv \
    -- python3 bench.py --no-cg --no-gamg --no-host-vec --no-flan --no-cpu-baseline > "$OUT/bench_headline_prof.json" \
    2> "$OUT/bench_headline_prof.err" && echo "headline prof ok" || { tail -20 "$OUT/bench_headline_prof.err"; exit 1; }
timeout -k 10 400 bash tools/gpu_pmc_case.sh "$TAG/pmc_codes" poisson --its 20 > "$OUT/pmc_codes.log" 2>&1 \
 && echo "pmc codes ok" && timeout -k 10 400 bash tools/gpu_pmc_case.sh "$TAG/pmc_aj" poisson --its 20 --opt column_codes=0 \
    > "$OUT/pmc_aj.log" 2>&1 && echo "pmc aj ok"
