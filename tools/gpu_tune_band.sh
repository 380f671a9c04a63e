#!/bin/bash
# x tiles for banded scattered gathers (geometries 9/10) on the skewed and
# FEM-structured stand-ins, plus the geometry parity tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-band}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "x_tile or speed_only or geometry" > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
 && timeout -k 10 300 python -u tools/tune.py --matrix skewed --variants xtile_band --rounds 3 > "$OUT/skewed.jsonl" 2>&1 \
 && timeout -k 10 300 python -u tools/tune.py --matrix skewed_nohub --variants xtile_band --rounds 3 > "$OUT/skewed_nohub.jsonl" 2>&1 \
 && timeout -k 10 300 python -u tools/tune.py --matrix fem_hex --variants xtile_band --rounds 3 > "$OUT/fem.jsonl" 2>&1 \
 && grep us_median "$OUT"/*.jsonl
rc=$?; [ $rc -ne 0 ] && tail -30 "$OUT/pytest.log"; exit $rc
