#!/bin/bash
# Round 3 closing record: the whole GPU suite, the driver's default bench
# line, rocprofv3 kernel statistics of the headline-only bench (the STREAM
# kernel the roofline block names) and of the full bench (solver and set-up
# kernels), and the HBM-traffic PMC passes of the 300^3 SpMV.
set -o pipefail
TAG=${1:-r03z}
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
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-host-vec > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
    && echo "full prof ok" || { tail -20 "$OUT/bench_prof.err"; exit 1; }
timeout -k 10 400 bash tools/gpu_pmc_case.sh "$TAG/pmc_poisson" poisson --its 20 > "$OUT/pmc.log" 2>&1 \
    && echo "pmc ok" && tail -3 "$OUT/pmc.log"
