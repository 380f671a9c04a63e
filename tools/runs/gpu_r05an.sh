#!/bin/bash
# Round 5: the bench with the stand-ins' live PMC traffic (no CG / GAMG legs).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05an
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --no-cg --no-gamg --no-host-vec > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); f=d['flan_standin']
print('headline traffic', d['roofline']['traffic'])
for n in ('skewed','fem_hex'):
    r=f[n]['stream']; print(n, r.get('us_mean'), r.get('layout_bytes'), r.get('traffic'), r.get('traffic_vs_layout_bytes'), r.get('traffic_detail'))"
