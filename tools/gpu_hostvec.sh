#!/bin/bash
# Host-vector MatMult: parity tests, then the bench's host_vec / CPU lines only.
set -o pipefail
TAG=${1:-hostvec}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -k "mult_host" > "$OUT/pytest.log" 2>&1 \
 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
 && timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cg --no-gamg > "$OUT/bench.json" 2> "$OUT/bench.err" \
 && echo "bench ok" && python -c "import json;d=json.load(open('$OUT/bench.json'));print(json.dumps(d['host_vec']));print(d['cpu_baseline_all_cores'])"
rc=$?
[ $rc -ne 0 ] && tail -40 "$OUT/pytest.log" && tail -20 "$OUT/bench.err" 2>/dev/null
exit $rc
