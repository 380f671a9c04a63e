#!/bin/bash
# N = 8 projection parts on one GPU, the zero-ghost overhead under the
# profiler, and the LDS-DMA read shapes.
set -o pipefail
TAG=${1:-r03e}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
true
true
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for P in 37 38 300; do
  timeout -k 10 300 python3 -u tools/slab_probe.py --planes $P > "$OUT/slab_$P.json" 2> "$OUT/slab_$P.err" || { tail -20 "$OUT/slab_$P.err"; exit 1; }
  cat "$OUT/slab_$P.json"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_slab" -o run --output-format csv -- python3 tools/slab_probe.py --planes 37 \
    > "$OUT/prof_slab.log" 2>&1 && echo "prof ok" || { tail -20 "$OUT/prof_slab.log"; exit 1; }
