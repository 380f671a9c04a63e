#!/bin/bash
# Round 5: kernel statistics of the skewed stand-in, hub segments after the
# row blocks (serial) — the segment kernel's own duration.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05x
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
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
