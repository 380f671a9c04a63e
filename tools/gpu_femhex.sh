#!/bin/bash
# FEM-structured Flan_1565 stand-in: parity tests, then kernel/geometry sweep.
set -o pipefail
TAG=${1:-femhex}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_harness.py -x -q --timeout 120 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
    || { tail -30 "$OUT/pytest.log"; exit 1; }
timeout -k 10 300 python -u tools/tune.py --matrix fem_hex --variants skewed --rounds 3 > "$OUT/tune_femhex.jsonl" 2>&1 \
    || { tail -20 "$OUT/tune_femhex.jsonl"; exit 1; }
grep us_median "$OUT/tune_femhex.jsonl"
timeout -k 10 300 python -u tools/tune.py --matrix fem_hex --variants xtile --rounds 3 > "$OUT/tune_femhex_xtile.jsonl" 2>&1 \
    || { tail -20 "$OUT/tune_femhex_xtile.jsonl"; exit 1; }
grep us_median "$OUT/tune_femhex_xtile.jsonl"
