# A/B of set-up / layout environment switches in the solver's context:
# CG + GAMG at 300^3 (tools/prof_case.py gamg) under a rocprofv3 kernel trace,
# one process per setting, then one FETCH_SIZE pass; summary:
# tools/tmpl_summary.py.   bash tools/runs/tmpl_ab.sh TAG "VAR=VAL ..." ...
set -o pipefail
OUT=gpurun_out/r06/${1:?tag}; shift; mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "$@"; do
  name=$(echo "$cfg" | tr ' =' '__')
  eval "$cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace_$name -o run --output-format csv -- python3 tools/prof_case.py gamg --grid 300 --solves 1" > $OUT/trace_$name.log 2>&1 || exit $?
  echo "$name: $(grep 'gamg: set-up' $OUT/trace_$name.log)"
done
