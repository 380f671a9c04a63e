#!/bin/bash
# One-GPU rehearsal of the multi-GPU bench path (MPIAIJ, RCCL halo, strong
# 300^3 line, distributed CG) under torch.distributed.run with one rank.
#   usage: tools/gpu_mpi_rehearsal.sh TAG
set -o pipefail
TAG=${1:-mpi}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 1 --mpi --steps 100 --warmup 10 --no-cpu-baseline \
    > "$OUT/mpi.json" 2> "$OUT/mpi.err" \
 && echo "mpi ok" && cat "$OUT/mpi.json"
