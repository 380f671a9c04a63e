#!/bin/bash
# Long-row XCD placement: parity test, interleaved A/B on the skewed stand-in,
# kernel stats of the default path.  usage: tools/gpu_longxcd.sh TAG
set -o pipefail
TAG=${1:-lx}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread \
    -k "long_row or skewed or options_do_not" > "$OUT/pytest.log" 2>&1 \
 && echo "pytest ok" \
 && timeout -k 10 300 python -u tools/tune.py --matrix skewed --variants longxcd --rounds 7 > "$OUT/tune.jsonl" 2>&1 \
 && echo "tune ok" && grep us_median "$OUT/tune.jsonl" \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/skewed" -o run --output-format csv \
    -- python3 tools/prof_case.py skewed > "$OUT/skewed.log" 2>&1 \
 && echo "prof ok"
rc=$?
tail -3 "$OUT/pytest.log"
exit $rc
