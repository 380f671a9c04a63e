#!/bin/bash
# Wide blocks in the 16-bit gather-ordered launch: the SpMV parity tests, then
# the skewed / FEM stand-ins (gather-sort variants; hub segments serial vs on
# a side stream) and a kernel-trace of the skewed default.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/${1:-r03aa}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_flan_standins_gpu.py > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { tail -30 "$OUT/pytest.log"; exit 1; }
run() {  # matrix variants
  timeout -k 10 300 python3 tools/tune.py --matrix $1 --variants $2 --rounds 3 > "$OUT/$2_$1.jsonl" 2>&1 || { tail -20 "$OUT/$2_$1.jsonl"; return 1; }
  echo "== $1 $2"; python3 -c "
import json
rows=[json.loads(l) for l in open('$OUT/$2_$1.jsonl') if l.startswith('{')]
eq={r['variant']:(r['bitwise_equal_first'],r['max_abs_diff']) for r in rows if 'bitwise_equal_first' in r}
for d in sorted((r for r in rows if 'us_median' in r), key=lambda d: d['us_median']): print(round(d['us_median'],1), d['variant'], eq.get(d['variant'],''))"
}
run skewed gsort && run skewed gslong && run fem_hex gsort && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_skewed" -o run --output-format csv \
    -- python3 tools/prof_case.py skewed --its 20 > "$OUT/prof_skewed.log" 2>&1 && echo "prof ok" && \
python3 -c "
import csv,glob
f=glob.glob('$OUT/prof_skewed/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]: print(r['Name'][:110], r['Calls'], r['AverageNs'])"
