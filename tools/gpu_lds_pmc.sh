#!/bin/bash
# SQ counters (LDS bank conflicts, wave-cycle split) of the STREAM kernel on
# the skewed stand-in and on 300^3 Poisson, one rocprofv3 --pmc pass each.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-ldspmc}
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
for c in skewed poisson; do
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/$c" -o run \
      -- python3 tools/prof_case.py $c --its 20 > "$OUT/$c.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for c in ("skewed", "poisson"):
    f = glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for row in csv.DictReader(open(f[0])):
        k = row["Kernel_Name"][:60]
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        n[(k, row["Counter_Name"])] += 1
    for k, d in acc.items():
        if "stream" not in k and "long" not in k:
            continue
        calls = max(n[(k, "SQ_WAVE_CYCLES")], 1)
        print(c, k, {m: round(v / calls) for m, v in sorted(d.items())})
PY
