#!/bin/bash
# The multi-rank GPU tests (unfused-dot case added), geometries 9-11 on the
# configs[4] stand-ins, then the set-up breakdown.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-r03o}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread tests/test_mpi_gpu.py \
    > "$OUT/pytest_mpi.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest_mpi.log")" \
 && timeout -k 10 300 python3 tools/tune.py --matrix skewed --variants skewgeom2 --rounds 3 > "$OUT/skewgeom2.jsonl" 2>&1 \
 && timeout -k 10 300 python3 tools/tune.py --matrix skewed_nohub --variants skewgeom2 --rounds 3 > "$OUT/skewgeom2_nohub.jsonl" 2>&1 \
 && timeout -k 10 300 python3 tools/tune.py --matrix fem_hex --variants skewgeom2 --rounds 3 > "$OUT/skewgeom2_fem.jsonl" 2>&1 \
 && AIJHIP_GAMG_LOG=1 timeout -k 10 300 python -u tools/prof_case.py gamg > "$OUT/setup_hash.log" 2>&1 \
 && for f in "$OUT"/skewgeom2*.jsonl; do echo "== $f"; grep us_median "$f" | python3 -c "
import sys,json
r=[json.loads(l) for l in sys.stdin]
for d in sorted(r,key=lambda d:d['us_median']): print(round(d['us_median'],1), d['variant'])"; done
