#!/bin/bash
# Round 5: long rows after the row blocks by default — parity tests, the
# skewed A/B (default vs side stream), the bench's stand-in legs.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05ae
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python -u -m pytest tests/test_flan_standins_gpu.py tests/test_gpu_parity.py -x -q -m gpu \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/ab_opts.py --case skewed --variant '{}' --variant '{"long_overlap": 1}' \
    > "$OUT/ab_skewed.jsonl" 2> "$OUT/ab_skewed.err" || { tail -20 "$OUT/ab_skewed.err"; exit 1; }
cat "$OUT/ab_skewed.jsonl"
timeout -k 10 400 python -u bench.py --no-cg --no-gamg --no-host-vec --no-cpu-baseline --no-pmc > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); f=d['flan_standin']
print('bench headline', d['roofline']['kernel_us_mean'], {k:(v.get('us_mean'), v.get('long_overlap')) for k,v in f['skewed'].items() if isinstance(v,dict) and 'us_mean' in v})"
