#!/bin/bash
# Round 5: kernel statistics of the PETSc-MIS GAMG set-up + solve (300^3).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05k
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mis" -o run --output-format csv \
    -- python3 -u tools/prof_case.py gamg --gamg-opt coarsen=1 --gamg-opt eig_ksp=1 > "$OUT/mis.log" 2>&1 \
    || { tail -30 "$OUT/mis.log"; exit 1; }
grep -E "gamg: set-up" "$OUT/mis.log"
f=$(find "$OUT/prof_mis" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:40]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:10.1f} us  {r["Name"][:110]}')
PY
