#!/bin/bash
# Round 5 closing record, part 2: the N = 8 one-GPU rehearsal, rocprofv3
# kernel statistics of the whole bench, SQ wait / issue counters of the
# skewed stand-in and the headline operand.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ag
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --gpus 8 --rehearse-one-gpu --grid 100 --strong-grid 300 --steps 20 \
    --warmup 3 > "$OUT/bench_rehearse_n8.json" 2> "$OUT/bench_rehearse_n8.err" \
    && echo "rehearsal n8 ok" || { tail -20 "$OUT/bench_rehearse_n8.err"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-host-vec > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
    && echo "full prof ok" || { tail -20 "$OUT/bench_prof.err"; exit 1; }
bash tools/pmc_sq.sh r05ag/sq skewed poisson
