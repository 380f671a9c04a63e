# Counters of the row-template MatMult beside the CSR one at 300^3
# (tools/prof_case.py poisson, automatic layout / PETSc's CSR): SQ wait and
# issue, then TA / TD busy, L1 and L2 requests, one rocprofv3 --pmc pass each.
#   bash tools/runs/tmpl_pmc.sh TAG
set -o pipefail
OUT=gpurun_out/r06/${1:?tag}; mkdir -p $OUT
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES"
MEM="TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
for lay in auto csr; do
  opts=""; mkdir -p $OUT/$lay
  [ $lay = csr ] && opts="--opt row_templates=0 --opt row_patterns=0 --opt column_codes=0"
  timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/$lay/trace -o run --output-format csv \
    -- python3 tools/prof_case.py poisson --its 10 $opts > $OUT/$lay/trace.log 2>&1 || exit 1
  i=0
  for C in "$SQ" "$MEM"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $C -d $OUT/$lay/pmc$i -o run --output-format csv \
      -- python3 tools/prof_case.py poisson --its 10 $opts > $OUT/$lay/pmc$i.log 2>&1 || exit 1
  done
  python3 tools/pmc_summary.py $OUT/$lay > $OUT/$lay/summary.json || exit 1
  echo "$lay ok"
done
