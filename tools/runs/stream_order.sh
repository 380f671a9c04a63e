# the skewed stand-in's stream-order swing. Kernel traces
# of tools/ab_opts.py --case skewed with 0 and 1 dummy streams created before
# the matrices, alternating, two each; summary: tools/stream_order_summary.py.
set -o pipefail
OUT=gpurun_out/r06/${1:?tag}; mkdir -p $OUT
export TMPDIR=/tmp
for k in 0 1 0 1; do
  n=$((${n:-0} + 1))
  timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/trace_${n}_k$k -o run --output-format csv -- python3 tools/ab_opts.py --case skewed --dummy-streams $k --rounds 10 > $OUT/ab_${n}_k$k.log 2>&1 || exit $?
  echo "run $n dummy-streams $k: $(grep '^{' $OUT/ab_${n}_k$k.log | cut -c1-160)"
done
