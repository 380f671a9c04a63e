#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/s9
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/tune.py --matrix banded --variants rel --rounds 5 > "$OUT/rel_banded.jsonl" 2>&1 \
  && grep -h "bitwise\|us_median" "$OUT/rel_banded.jsonl" | cut -c1-200 || exit 1
timeout -k 10 300 python -u tools/tune.py --matrix skewed --variants rel --rounds 4 > "$OUT/rel_skewed.jsonl" 2>&1 \
  && grep -h "us_median" "$OUT/rel_skewed.jsonl" | cut -c1-200 || exit 1
timeout -k 10 300 python -u tools/tune.py --matrix fem_hex --variants rel --rounds 3 > "$OUT/rel_fem.jsonl" 2>&1 \
  && grep -h "us_median" "$OUT/rel_fem.jsonl" | cut -c1-200 || exit 1
