#!/bin/bash
# Round-3 closing record: the GPU suite, smoke(), the default bench line, and
# rocprofv3 kernel statistics of the headline alone and of the whole bench.
#   usage: tools/gpu_r03final.sh TAG
set -o pipefail
TAG=${1:-r03final}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || { tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_headline" -o run --output-format csv \
    -- python3 bench.py --no-cg --no-gamg --no-host-vec --no-flan --no-cpu-baseline > "$OUT/bench_headline_prof.json" \
    2> "$OUT/bench_headline_prof.err" && echo "headline prof ok" || { tail -20 "$OUT/bench_headline_prof.err"; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-host-vec > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
    && echo "full prof ok" || { tail -20 "$OUT/bench_prof.err"; exit 1; }
