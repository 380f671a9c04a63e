#!/bin/bash
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
OUT=$ROOT/gpurun_out/r02d
mkdir -p "$OUT"
tools/gpu_mpi.sh r02d_mpi && timeout -k 10 300 python -u bench.py --steps 50 --no-cg --no-gamg --no-host-vec \
   --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" && python3 -c "
import json;d=json.load(open('$OUT/bench.json'));print(d['roofline'])"
