#!/bin/bash
# After column codes and the MERGE load rewrite: the GPU suite, the default
# bench line, and one-process timings of STREAM / MERGE on the skewed stand-in.
#   usage: tools/gpu_r03c.sh TAG
set -o pipefail
TAG=${1:-r03c}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
echo "bench ok"
timeout -k 10 300 python -u tools/tune.py --variants merge --matrix skewed --rounds 3 --launches 20 > "$OUT/tune_merge_skewed.jsonl" 2>&1 || { tail -5 "$OUT/tune_merge_skewed.jsonl"; exit 1; }
grep us_median "$OUT/tune_merge_skewed.jsonl"
timeout -k 10 300 python -u tools/tune.py --variants merge --matrix fem_hex --rounds 3 --launches 20 > "$OUT/tune_merge_fem.jsonl" 2>&1 || { tail -5 "$OUT/tune_merge_fem.jsonl"; exit 1; }
grep us_median "$OUT/tune_merge_fem.jsonl"
