#!/bin/bash
# Gather-ordered row blocks: the SpMV parity tests (full-size configs[4]
# stand-ins included), then sorted vs unsorted on the stand-ins and 300^3.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-r03w}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_flan_standins_gpu.py > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { tail -30 "$OUT/pytest.log"; exit 1; }
for mtx in skewed skewed_nohub fem_hex poisson; do
  timeout -k 10 300 python3 tools/tune.py --matrix $mtx --variants gsort --rounds 3 > "$OUT/gsort_$mtx.jsonl" 2>&1 || { tail -20 "$OUT/gsort_$mtx.jsonl"; exit 1; }
  echo "== $mtx"; python3 -c "
import json
rows=[json.loads(l) for l in open('$OUT/gsort_$mtx.jsonl') if l.startswith('{')]
eq={r['variant']:(r['bitwise_equal_first'],r['max_abs_diff']) for r in rows if 'bitwise_equal_first' in r}
for d in sorted((r for r in rows if 'us_median' in r), key=lambda d: d['us_median']): print(round(d['us_median'],1), d['variant'], eq.get(d['variant'],''))"
done
