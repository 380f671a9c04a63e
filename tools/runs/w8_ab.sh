# The pipelined template kernel at its natural register count vs forced to
# 8 waves per SIMD (__launch_bounds__(512, 8); some epilogues then spill a
# few words), alternating, each a bench without the stand-in / host-vector /
# PMC legs: CG + Jacobi it/s and the CG + GAMG solve.
set -o pipefail
OUT=gpurun_out/r06/${1:?tag}; mkdir -p $OUT
n=0
for w in 0 1 0 1; do
  n=$((n + 1))
  AIJHIP_TMPL_W8=$w timeout -k 10 300 python -u bench.py --no-flan --no-host-vec --no-pmc --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_${n}_w$w.json 2> $OUT/bench_${n}_w$w.err || exit $?
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$OUT/bench_${n}_w$w.json') if l.startswith('{')][-1]; print('w8=$w', d['cg']['iters_per_s'], d['cg_gamg']['solve_s'], d['effective']['us_mean'])"
done
