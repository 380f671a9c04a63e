#!/bin/bash
# Round 3 closing record (after the gather-ordered blocks): the GPU suite,
# the driver's default bench line, rocprofv3 kernel statistics (headline-only
# and full bench), and the skewed stand-in's SQ wait counters and HBM traffic.
set -o pipefail
TAG=${1:-r03z2}
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
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/sq_skewed" -o run \
    -- python3 tools/prof_case.py skewed --its 20 > "$OUT/sq_skewed.log" 2>&1 && echo "sq ok" \
 && timeout -k 10 400 bash tools/gpu_pmc_case.sh "$TAG/pmc_skewed" skewed --its 20 > "$OUT/pmc_skewed.log" 2>&1 \
 && echo "pmc skewed ok" && tail -3 "$OUT/pmc_skewed.log"
