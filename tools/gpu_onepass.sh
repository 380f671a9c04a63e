#!/bin/bash
# One-pass Galerkin product: GAMG/KSP GPU tests, A/B of the set-up in
# alternating processes, and the per-phase set-up log of both forms.
#   usage: tools/gpu_onepass.sh TAG
set -o pipefail
TAG=${1:-onepass}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gamg.py tests/test_ksp.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/gpu_ab_env.sh "$TAG" AIJHIP_ROWPROD_ONE_PASS 0 1 2 || exit 1
for v in 0 1; do
  AIJHIP_GAMG_LOG=1 AIJHIP_ROWPROD_ONE_PASS=$v timeout -k 10 200 python -u tools/prof_case.py gamg \
      > "$OUT/log_$v.txt" 2>&1 || exit 1
  echo "ONE_PASS=$v"; grep -E "A\*P|P\^T\*|gamg: set-up" "$OUT/log_$v.txt" | tail -9
done
