#!/bin/bash
# The device-resident emax power iteration: the GAMG GPU tests (device
# hierarchy bitwise against the host builder, 300^3 included), then the
# set-up breakdown and CG+GAMG timings (tools/prof_case.py gamg, twice).
#   usage: tools/gpu_emax.sh TAG
set -o pipefail
TAG=${1:-emax}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gamg.py tests/test_solver_configs.py -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { grep -E "FAIL|Error|assert" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
for r in 1 2; do
  AIJHIP_GAMG_LOG=1 timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_$r.log" 2>&1 || { tail -20 "$OUT/gamg_$r.log"; exit 1; }
  grep -E "gamg: |emax|level 0 phase 1 |level 1 phase 1 " "$OUT/gamg_$r.log" | head -20
done
