#!/bin/bash
# Round 5: the deferred-RCCL halo (halo_finish enqueues the collective), the
# device-only / pipelined halo probe, the MPI + GAMG GPU tests it touches,
# PETSc's MIS coarsening on the device, and the buffer-load phase-1 A/B.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05b
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rccl_selfhalo_gpu.py tests/test_mpi_gpu.py tests/test_comm_gpu.py \
    tests/test_gamg.py tests/test_abi.py -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u -m pytest tests/test_solver_configs.py -x -v -m gpu -k mis --timeout 300 \
    --timeout-method thread > "$OUT/pytest_mis.log" 2>&1 || { tail -30 "$OUT/pytest_mis.log"; exit 1; }
grep -E "MIS hierarchy|passed|failed" "$OUT/pytest_mis.log"
for mat in poisson fem_hex; do
  timeout -k 10 200 python -u tools/ab_buf.py --matrix $mat >> "$OUT/ab_buf.jsonl" 2> "$OUT/ab_buf_$mat.err" \
      || { tail -20 "$OUT/ab_buf_$mat.err"; exit 1; }
done
cat "$OUT/ab_buf.jsonl"
timeout -k 10 300 python -u tools/halo_probe.py --grid 300 --planes 300 38 --reps 200 > "$OUT/halo.jsonl" 2> "$OUT/halo.err" \
    || { tail -20 "$OUT/halo.err"; exit 1; }
cat "$OUT/halo.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d "$OUT/trace" -o run \
    -- python3 tools/halo_probe.py --grid 300 --planes 38 --reps 20 --burst 20 --only diag,forkjoin,ag_empty,p2p_selfd,p2p_self \
    > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
echo trace ok
