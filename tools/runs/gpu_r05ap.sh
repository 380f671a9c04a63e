#!/bin/bash
# Round 5: does the side stream's result follow its hardware queue? The
# skewed default vs side stream after 0..7 other streams were created.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ap
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
for k in 0 1 2 3 5 7; do
  timeout -k 10 300 python -u tools/ab_opts.py --case skewed --rounds 20 --dummy-streams $k \
      --variant '{}' --variant '{"long_overlap": 1}' > "$OUT/ab_k$k.jsonl" 2> "$OUT/ab_k$k.err" \
      || { tail -20 "$OUT/ab_k$k.err"; exit 1; }
  echo "k $k: $(python3 -c "
import json,sys; r=[json.loads(l) for l in open('$OUT/ab_k$k.jsonl')]; print(' / '.join('%s %.1f' % (x['options'], x['us_median']) for x in r))")"
done
