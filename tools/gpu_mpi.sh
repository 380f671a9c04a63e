#!/bin/bash
# Native row-partitioned path on one GPU: the MPI/KSP GPU tests, then the
# N = 1 --mpi rehearsal over RCCL and an N = 2 rehearsal over the host
# transport (ranks share cuda:0). Every GPU step has its own time limit.
#   usage: tools/gpu_mpi.sh TAG
set -o pipefail
TAG=${1:-mpi}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_comm_gpu.py tests/test_mpi_gpu.py tests/test_ksp.py tests/test_ksp_mpi.py > "$OUT/pytest.log" 2>&1 \
 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
 && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 1 --mpi --steps 50 --warmup 5 --no-cpu-baseline --no-strong \
      > "$OUT/bench_mpi_n1.json" 2> "$OUT/bench_mpi_n1.err" \
 && echo "mpi n1 ok" && cat "$OUT/bench_mpi_n1.json" \
 && timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29512 bench.py --gpus 2 --rehearse-one-gpu --grid 160 --steps 20 --warmup 3 --cg-iters 50 \
      > "$OUT/bench_rehearse_n2.json" 2> "$OUT/bench_rehearse_n2.err" \
 && echo "rehearse n2 ok" && cat "$OUT/bench_rehearse_n2.json"
rc=$?
[ $rc -ne 0 ] && tail -40 "$OUT/pytest.log" && tail -20 "$OUT"/*.err 2>/dev/null
exit $rc
