#!/bin/bash
# Round 5: CG vector kernels two elements per lane — CG tests, then the
# bench's CG legs (headline for the box's scale).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05v
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ksp.py tests/test_solver_configs.py -x -q -m gpu \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py --no-flan --no-host-vec --no-cpu-baseline --no-pmc > "$OUT/bench_$rep.json" \
      2> "$OUT/bench_$rep.err" || { tail -20 "$OUT/bench_$rep.err"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$rep.json').read().strip().splitlines()[-1])
print('headline us', d['roofline']['kernel_us_mean'], 'cg it/s', d['cg']['iters_per_s'], 'gamg', d['cg_gamg']['solve_s'], d['cg_gamg']['setup_again_s'], d['cg_gamg'].get('hierarchy_comparison'))"
done
