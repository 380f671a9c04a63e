#!/bin/bash
# Round 5: kernel traces of CG + GAMG at 300^3 with the set-up's operators
# unsorted (0), gather-ordered (1) and automatic (-1: sorted where the 16-bit
# form fits), then the automatic form's timing beside the other two.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05as
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
for g in 0 1 -1; do
  AIJHIP_SETUP_GSORT=$g timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_g$g" -o run \
      -- python3 -u tools/prof_case.py gamg > "$OUT/trace_g$g.log" 2>&1 || { tail -20 "$OUT/trace_g$g.log"; exit 1; }
  grep -E '^gamg' "$OUT/trace_g$g.log"
done
for g in -1 0 1 -1; do
  AIJHIP_SETUP_GSORT=$g timeout -k 10 240 python -u tools/prof_case.py gamg --solves 3 > "$OUT/gamg_g$g.log" 2>&1 \
    || { tail -20 "$OUT/gamg_g$g.log"; exit 1; }
  echo "gsort $g: $(grep -E '^gamg' "$OUT/gamg_g$g.log" | tr '\n' ' ')"
done
