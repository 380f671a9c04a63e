# Row-template kernel A/B in the solver's context: CG + GAMG at 300^3
# (tools/prof_case.py gamg) under a rocprofv3 kernel trace, one process per
# setting (the knobs are read once per process), then one FETCH_SIZE pass.
#   bash tools/runs/tmpl_ab.sh TAG "PIPE SPLIT" ...
set -o pipefail
OUT=gpurun_out/r06/${1:?tag}; shift; mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "$@"; do
  set -- $cfg
  name=p$1_s$2
  AIJHIP_TMPL_PIPE=$1 AIJHIP_TMPL_SPLIT=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace_$name -o run --output-format csv -- python3 tools/prof_case.py gamg --grid 300 --solves 1 > $OUT/trace_$name.log 2>&1 || exit $?
  echo "$name: $(grep 'gamg: set-up' $OUT/trace_$name.log)"
  AIJHIP_TMPL_PIPE=$1 AIJHIP_TMPL_SPLIT=$2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$name -o run -- python3 tools/prof_case.py gamg --grid 300 --solves 1 > $OUT/fetch_$name.log 2>&1 || exit $?
done
