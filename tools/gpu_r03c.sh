#!/bin/bash
# Distributed GAMG: GPU tests (k ranks on one GPU over the host transport),
# the refactored single-GPU set-up's bitwise tests, then bench.py's N = 2 and
# N = 4 weak-scaling rehearsals (300^3 rows per rank) for the iteration count.
set -o pipefail
TAG=${1:-r03c}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gamg_mpi_gpu.py tests/test_mpi_gpu.py tests/test_comm_gpu.py \
    tests/test_gamg.py tests/test_solver_configs.py -x -v -s -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" || { grep -E "PASS|FAIL|Error|error|its" "$OUT/pytest.log" | tail -40; exit 1; }
grep -E "ranks|its" "$OUT/pytest.log" | head -20
AIJHIP_GAMG_LOG=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29521 bench.py --gpus 2 --rehearse-one-gpu --steps 5 --warmup 2 --cg-iters 10 --no-strong \
    > "$OUT/n2.json" 2> "$OUT/n2.err" && echo "n2 ok" && python3 -c "
import json;d=json.loads(open('$OUT/n2.json').read().strip().splitlines()[-1]);print(json.dumps(d.get('cg_gamg')))" || { tail -30 "$OUT/n2.err"; exit 1; }
timeout -k 10 700 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29522 bench.py --gpus 4 --rehearse-one-gpu --steps 5 --warmup 2 --cg-iters 10 --no-strong \
    > "$OUT/n4.json" 2> "$OUT/n4.err" && echo "n4 ok" && python3 -c "
import json;d=json.loads(open('$OUT/n4.json').read().strip().splitlines()[-1]);print(json.dumps(d.get('cg_gamg')))" || { tail -30 "$OUT/n4.err"; exit 1; }
