#!/bin/bash
# Row patterns: 16-B vs 8-B LDS pair writes (AIJHIP_PAT_W16) at 300^3.
#   usage: tools/gpu_patw16.sh TAG
set -o pipefail
TAG=${1:-patw16}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_row_patterns_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { tail -20 "$OUT/pytest.log"; exit 1; }
timeout -k 10 400 python -u tools/tune.py --variants patw16 --rounds 5 --launches 20 > "$OUT/tune_poisson.jsonl" 2>&1 || { tail -5 "$OUT/tune_poisson.jsonl"; exit 1; }
grep -E "us_median|bitwise" "$OUT/tune_poisson.jsonl"
