set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES"
for case in skewed_nohub poisson; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/sq/$case -o run --output-format csv -- python3 tools/prof_case.py $case --its 10 --exact 1 > gpurun_out/sq/$case.log 2>&1 || exit 1
done
echo done
