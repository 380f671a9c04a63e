#!/bin/bash
# Round 5, first GPU call: the CSR-layout full-size parity legs, the
# interleaved halo probe (tools/halo_probe.py) and a kernel + HIP API trace
# of the one-rank distributed MatMult forms.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05a
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread \
    -k "full_size or max_size_600" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/halo_probe.py --grid 300 --planes 300 38 --reps 200 > "$OUT/halo.jsonl" 2> "$OUT/halo.err" \
    || { tail -20 "$OUT/halo.err"; exit 1; }
cat "$OUT/halo.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d "$OUT/trace" -o run \
    -- python3 tools/halo_probe.py --grid 300 --planes 38 --reps 20 --only diag,forkjoin,ag_empty,p2p_selfd,p2p_self \
    > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
echo trace ok
