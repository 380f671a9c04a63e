#!/bin/bash
# pytest -m gpu, then the 300^3 CSR block-shape A/B (tune.py geo3) and the
# skewed stand-in's launch forms (tools/gpu_skewed.sh). Chained: the first
# failure ends the call.
#   usage: tools/gpu_s2.sh TAG
set -o pipefail
TAG=${1:-s2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
    && tail -1 "$OUT/pytest.log" || { tail -20 "$OUT/pytest.log"; exit 1; }
timeout -k 10 300 python -u tools/tune.py --variants geo3 --rounds 3 > "$OUT/geo3.jsonl" 2>&1 \
    && echo "geo3 ok" && grep -h "us_median" "$OUT/geo3.jsonl" | tail -7 || exit 1
bash tools/gpu_skewed.sh "$TAG/skewed"
