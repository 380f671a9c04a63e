#!/bin/bash
# Round 5: wide blocks on the branch-free NT phase 1 — stand-in parity tests,
# the skewed A/B (side stream vs serial), kernel statistics (serial).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05y
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python -u -m pytest tests/test_flan_standins_gpu.py tests/test_gpu_parity.py -x -q -m gpu \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/ab_opts.py --case skewed \
    --variant '{}' --variant '{"long_overlap": 0}' > "$OUT/ab_skewed.jsonl" 2> "$OUT/ab_skewed.err" \
    || { tail -20 "$OUT/ab_skewed.err"; exit 1; }
cat "$OUT/ab_skewed.jsonl"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_serial" -o run --output-format csv \
    -- python3 tools/prof_case.py skewed --its 20 --opt long_overlap=0 > "$OUT/serial.log" 2>&1 \
    || { tail -20 "$OUT/serial.log"; exit 1; }
python3 - "$OUT/prof_serial/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    print(f'{int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:120]}')
PY
