#!/bin/bash
# Round 3 record: the whole GPU suite, the bench line (50 timed steps) and
# its kernel statistics, the skewed stand-in's kernel trace and SQ counters.
set -o pipefail
TAG=${1:-r03f}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
timeout -k 10 500 python -u bench.py --steps 50 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
echo "bench ok"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv \
    -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-host-vec > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
    && echo "prof ok" || { tail -20 "$OUT/bench_prof.err"; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/sq_skewed" -o run \
    -- python3 tools/prof_case.py skewed --its 20 > "$OUT/sq_skewed.log" 2>&1 && echo "sq ok" && timeout -k 10 300 python3 tools/tune.py --matrix skewed --variants skewgeom --rounds 3 > "$OUT/skewgeom.jsonl" 2>&1 && grep us_median "$OUT/skewgeom.jsonl" | head -8
