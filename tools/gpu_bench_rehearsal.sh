#!/bin/bash
# bench.py's N > 1 code path rehearsed on a one-GPU box: N ranks on cuda:0
# over gloo (RCCL refuses two ranks on one device). Checks control flow and
# the JSON line, not scaling.
#   usage: tools/gpu_bench_rehearsal.sh TAG
set -o pipefail
TAG=${1:-rehearse}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29521 bench.py --gpus 2 --rehearse-one-gpu --steps 20 --warmup 3 --cg-iters 20 \
    > "$OUT/n2_p2p.json" 2> "$OUT/n2_p2p.err" && echo "n2 ok" && cat "$OUT/n2_p2p.json" \
 && timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29522 bench.py --gpus 4 --rehearse-one-gpu --halo allgather --steps 10 --warmup 2 --cg-iters 10 \
    > "$OUT/n4_allgather.json" 2> "$OUT/n4_allgather.err" && echo "n4 ok" && cat "$OUT/n4_allgather.json"
rc=$?
[[ $rc != 0 ]] && tail -30 "$OUT"/*.err
exit $rc
