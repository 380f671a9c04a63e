#!/bin/bash
# Counters of the CSR MatMult (aj read) at 300^3: kernel trace + HBM traffic
# passes (tools/gpu_pmc_case.sh), then the SQ wait / issue pass and an L1
# (TCP) pass, each its own rocprofv3 run (no --pmc beside trace domains).
#   usage: tools/gpu_pmc_csr.sh TAG
set -o pipefail
TAG=${1:-pmccsr}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
CASE="poisson --its 20 --opt row_patterns=0 --opt column_codes=0"
bash tools/gpu_pmc_case.sh "$TAG" $CASE > "$OUT/case.log" 2>&1 && echo "traffic ok" \
 && timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
      SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/sq" -o run \
      -- python3 tools/prof_case.py $CASE > "$OUT/sq.log" 2>&1 && echo "sq ok" \
 && timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES --output-format csv \
      -d "$OUT/lds" -o run -- python3 tools/prof_case.py $CASE > "$OUT/lds.log" 2>&1 && echo "lds ok" \
 && timeout -k 10 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv \
      -d "$OUT/tcp" -o run -- python3 tools/prof_case.py $CASE > "$OUT/tcp.log" 2>&1 && echo "tcp ok"
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary_all.json" 2>/dev/null; tail -c 1500 "$OUT/summary_all.json"
