#!/bin/bash
# Round 5: the default bench line (interleaved stand-in legs, the like-for-
# like hierarchy comparison, live PMC traffic), then the eight-rank one-GPU
# rehearsal of the driver's N = 8 run (MIS default across ranks).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05q
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
echo "bench ok"
timeout -k 10 900 python -u bench.py --gpus 8 --rehearse-one-gpu --grid 100 --strong-grid 300 --steps 20 \
    --warmup 3 > "$OUT/bench_rehearse_n8.json" 2> "$OUT/bench_rehearse_n8.err" \
    && echo "rehearsal n8 ok" || { tail -20 "$OUT/bench_rehearse_n8.err"; exit 1; }
