#!/bin/bash
# Round 5: the hardware-queue effect on the headline and FEM operands (0 or 1
# stream created before the first launch), skewed repeated.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05aq
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
for k in 0 1 0 1; do
  for case in poisson fem_hex skewed; do
    if [ $case = poisson ]; then v='{"row_patterns": 0, "column_codes": 0}'; else v='{}'; fi
    timeout -k 10 300 python -u tools/ab_opts.py --case $case --rounds 15 --dummy-streams $k --variant "$v" \
        > "$OUT/ab_${case}_k$k.jsonl" 2> "$OUT/ab_${case}_k$k.err" || { tail -20 "$OUT/ab_${case}_k$k.err"; exit 1; }
    echo "k $k $case: $(python3 -c "
import json; r=[json.loads(l) for l in open('$OUT/ab_${case}_k$k.jsonl')]; print(' / '.join('%.1f' % x['us_median'] for x in r))")"
  done
done
