#!/bin/bash
# Round-6 GPU-box records: one mode per call, each writing gpurun_out/r06/<tag>/
# (copied to profiles/r06/<tag>/ when kept). Every GPU step has its own time
# limit and the steps are chained, so the first failure ends the call.
#   usage: bash tools/runs/r06.sh MODE TAG
#   mpi1        — the N > 1 path at its real per-rank size:
#                 N = 1 over RCCL through torch.distributed.run with the
#                 distributed GAMG builder forced (AIJHIP_GAMG_DIST=1: 27 M rows
#                 on one rank)
#   rehearse_n2 — --gpus 2 --rehearse-one-gpu at 300^3 with CG + GAMG (13.5 M
#                 rows per rank, host transport)
#   default    — the driver's N = 1 command (python bench.py)
#   rehearse_n8 — the driver's N = 8 line on one GPU: 8 ranks over gloo (host
#                 transport), the 300^3 strong headline (38/37 planes), a 100^3
#                 weak block, distributed CG and CG + GAMG
#   tests      — pytest -m gpu + smoke()
#   final      — tests, then default, then the same bench under rocprofv3
#                --kernel-trace --stats (--no-pmc: counters need their own runs)
set -o pipefail
MODE=${1:?mode}; TAG=${2:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
if [ "$MODE" = final ]; then
  bash "$ROOT/tools/runs/r06.sh" tests "$TAG" && bash "$ROOT/tools/runs/r06.sh" default "$TAG" || exit 1
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
      -- python3 bench.py --no-pmc > "$OUT/bench_profiled.json" 2> "$OUT/bench_profiled.err" \
    && echo "profiled bench ok" || { tail -20 "$OUT/bench_profiled.err"; exit 1; }
  exit 0
fi
case $MODE in
  default)
    timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
      && echo "bench ok" || { tail -20 "$OUT/bench.err"; exit 1; }
    ;;
  mpi1)
    AIJHIP_GAMG_DIST=1 timeout -k 10 700 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --mpi --steps 20 --warmup 5 --wall-budget 600 \
        > "$OUT/bench_mpi_n1_gamgdist.json" 2> "$OUT/bench_mpi_n1_gamgdist.err" \
      && echo "mpi n1 ok" || { tail -20 "$OUT/bench_mpi_n1_gamgdist.err"; exit 1; }
    ;;
  rehearse_n2)
    timeout -k 10 1000 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --wall-budget 900 \
        > "$OUT/bench_rehearse_n2.json" 2> "$OUT/bench_rehearse_n2.err" \
      && echo "rehearsal n2 ok" || { tail -20 "$OUT/bench_rehearse_n2.err"; exit 1; }
    ;;
  rehearse_n8)
    timeout -k 10 1000 python -u bench.py --gpus 8 --rehearse-one-gpu --weak-grid 100 --steps 10 --warmup 3 \
        --wall-budget 900 > "$OUT/bench_rehearse_n8.json" 2> "$OUT/bench_rehearse_n8.err" \
      && echo "rehearsal n8 ok" || { tail -20 "$OUT/bench_rehearse_n8.err"; exit 1; }
    ;;
  tests)
    timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
        > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
      || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
      && tail -1 "$OUT/smoke.log" || { tail -20 "$OUT/smoke.log"; exit 1; }
    ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
esac
