#!/bin/bash
# Development checks on a GPU box (round 6): the distributed GAMG tests with
# the set-up log, the gather-ordered parity tests, and the single-GPU bench
# without the Flan / host-vector / PMC legs. A step that fails by a test
# (exit 1) lets the next run; any other failure (fault, abort, time limit)
# ends the call.
set -o pipefail
TAG=${1:?tag}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r06/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name: exit $rc ($(tail -1 "$OUT/$name.log" | cut -c1-150))"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
for s in ${STEPS:-gamg_mpi parity bench}; do
  case $s in
    gamg_mpi) AIJHIP_GAMG_LOG=1 step gamg_mpi 600 python -u -m pytest tests/test_gamg_mpi_gpu.py -x -v -s --timeout 300 --timeout-method thread ;;
    vcodes) step vcodes 400 python -u -m pytest tests/test_value_codes_gpu.py tests/test_gamg.py -x -v -m gpu --timeout 200 --timeout-method thread ;;
    patterns) step patterns 400 python -u -m pytest tests/test_row_patterns_gpu.py tests/test_ksp.py tests/test_solver_configs.py -x -v -m gpu --timeout 200 --timeout-method thread ;;
    parity) step parity 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "gather or geometry" --timeout 200 --timeout-method thread ;;
    bench) step bench 400 python -u bench.py --no-flan --no-host-vec --no-pmc --steps 20 --warmup 5 ;;
    tests) step tests 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ;;
    selfhalo) step selfhalo 300 python -u -m pytest tests/test_rccl_selfhalo_gpu.py tests/test_halo_errors_gpu.py -x -v --timeout 240 --timeout-method thread ;;
    graph) step graph_probe 300 python -u tools/graph_probe.py ;;
    graph_trace) step graph_trace 300 rocprofv3 --kernel-trace --hip-trace --stats -d "$OUT/graph_trace" -o run --output-format csv -- python3 tools/graph_probe.py --rounds 1 --its 160 ;;
  esac
done
