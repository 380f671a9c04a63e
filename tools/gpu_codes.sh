#!/bin/bash
# Column codes: their GPU tests, then one-process A/B timings (tools/tune.py
# --variants codes) on the 300^3 Poisson operand and the FEM stand-in.
#   usage: tools/gpu_codes.sh TAG
set -o pipefail
TAG=${1:-codes}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_column_codes_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
timeout -k 10 300 python -u tools/tune.py --variants codes --rounds 5 --launches 20 > "$OUT/tune_poisson.jsonl" 2>&1 || { tail -5 "$OUT/tune_poisson.jsonl"; exit 1; }
grep us_median "$OUT/tune_poisson.jsonl"
timeout -k 10 300 python -u tools/tune.py --variants codes --matrix fem_hex --rounds 5 --launches 20 > "$OUT/tune_fem.jsonl" 2>&1 || { tail -5 "$OUT/tune_fem.jsonl"; exit 1; }
grep us_median "$OUT/tune_fem.jsonl"
