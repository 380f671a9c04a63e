set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06/gs; mkdir -p $OUT
B="--opt row_templates=0 --opt row_patterns=0 --opt column_codes=0"
for cfg in "csr:$B --opt gather_sort=0" "sorted:$B --opt gather_sort=1"; do
  name=${cfg%%:*}; opts=${cfg#*:}
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/$name -o run --output-format csv -- python3 tools/prof_case.py poisson --its 20 $opts > $OUT/$name.log 2>&1 || exit 1
  grep -h "spmv" $OUT/$name/run_kernel_stats.csv | cut -c1-200
  grep -h "poisson" $OUT/$name.log | cut -c1-400
done
