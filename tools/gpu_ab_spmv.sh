#!/bin/bash
# A/B of two library builds on SpMV operands, alternating processes:
# tools/tune.py on each operand with the given variant set.
#   usage: tools/gpu_ab_spmv.sh TAG LIB_A LIB_B ROUNDS VARIANTS MATRIX...
set -o pipefail
TAG=$1; LA=$2; LB=$3; R=$4; V=$5; shift 5
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
for r in $(seq 1 "$R"); do
  for mat in "$@"; do
    for side in A B; do
      lib=$LA; [[ $side == B ]] && lib=$LB
      f="$OUT/${mat}_${side}_$r.jsonl"
      AIJHIP_AB=1 AIJHIP_LIB=$lib timeout -k 10 240 python -u tools/tune.py --matrix "$mat" --variants "$V" --rounds 3 > "$f" 2>&1 \
        || { tail -20 "$f"; exit 1; }
      echo "$mat $side r$r: $(python3 tools/tune_summary.py "$f")"
      grep -h '"bitwise_equal_first": false' "$f" | head -3
    done
  done
done
