#!/bin/bash
# Lane-stride (shuffled) gathers: parity, then A/B on the stand-ins and 300^3.
set -o pipefail
TAG=${1:-r03b}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread \
    -k "options or golden or skewed or row_group" > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { tail -40 "$OUT/pytest.log"; exit 1; }
for M in skewed skewed_nohub fem_hex poisson; do
  timeout -k 10 300 python -u tools/tune.py --matrix $M --variants shuf --rounds 3 > "$OUT/shuf_$M.jsonl" 2>&1 || exit 1
  grep -h "us_median\|bitwise" "$OUT/shuf_$M.jsonl" | grep -v "\"bitwise_equal_first\": true" | cut -c1-160
done
