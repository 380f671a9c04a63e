#!/bin/bash
# The N > 1 bench path after the set-up changes: N = 1 --mpi over RCCL (the
# real communicator; then with the distributed GAMG set-up forced at world
# size 1), and an N = 2 rehearsal over the host transport (ranks share cuda:0).
set -o pipefail
TAG=${1:-r03q}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 1 --mpi --steps 50 --warmup 5 --no-cpu-baseline --no-strong \
      > "$OUT/bench_mpi_n1.json" 2> "$OUT/bench_mpi_n1.err" \
 && echo "mpi n1 ok" \
 && AIJHIP_GAMG_DIST=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --mpi --steps 20 --warmup 3 --no-cpu-baseline \
      --no-strong > "$OUT/bench_mpi_n1_dist.json" 2> "$OUT/bench_mpi_n1_dist.err" \
 && echo "mpi n1 dist ok" \
 && timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29512 bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --cg-iters 10 \
      > "$OUT/bench_rehearse_n2.json" 2> "$OUT/bench_rehearse_n2.err" \
 && echo "rehearse n2 ok" \
 && for f in "$OUT"/bench_*.json; do python3 -c "
import json,sys
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
g=d.get('cg_gamg') or {}
print('$f'.split('/')[-1], d['value'], d['roofline']['frac'], 'cg', (d.get('cg') or {}).get('iters_per_s'), 'gamg its', g.get('its'), 'setup', g.get('setup_s'), 'solve', g.get('solve_s'), 'syncs', g.get('host_syncs'))"; done
rc=$?
[ $rc -ne 0 ] && tail -20 "$OUT"/*.err 2>/dev/null
exit $rc
