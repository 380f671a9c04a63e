#!/bin/bash
# Round 3, first GPU call: the GPU suite (row-group kernel, configs[4]
# full-size stand-ins, batched GAMG polling), the row-group A/B on the
# stand-ins, then the bench line with its Flan legs.
#   usage: tools/gpu_r03a.sh TAG
set -o pipefail
TAG=${1:-r03a}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { tail -40 "$OUT/pytest.log"; exit 1; }
for M in skewed skewed_nohub fem_hex; do
  timeout -k 10 240 python -u tools/tune.py --matrix $M --variants group --rounds 3 > "$OUT/group_$M.jsonl" 2>&1 || exit 1
  grep us_median "$OUT/group_$M.jsonl"
done
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
tail -c 3000 "$OUT/bench.json"
