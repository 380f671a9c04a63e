#!/bin/bash
# Record after row patterns: the GPU suite, the default bench line, rocprofv3
# kernel statistics of the headline alone, and the HBM-traffic PMC passes of
# 300^3 SpMVs with the automatic layout (row patterns).
#   usage: tools/gpu_r03p.sh TAG
set -o pipefail
TAG=${1:-r03p}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_headline" -o run --output-format csv \
    -- python3 bench.py --no-cg --no-gamg --no-host-vec --no-flan --no-cpu-baseline > "$OUT/bench_headline_prof.json" \
    2> "$OUT/bench_headline_prof.err" && echo "headline prof ok" || { tail -20 "$OUT/bench_headline_prof.err"; exit 1; }
timeout -k 10 400 bash tools/gpu_pmc_case.sh "$TAG/pmc_patterns" poisson --its 20 > "$OUT/pmc_patterns.log" 2>&1 \
 && echo "pmc patterns ok"
