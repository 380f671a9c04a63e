#!/bin/bash
# One GPU call that surveys the library after a change: the whole -m gpu
# suite, the GAMG set-up breakdown, an A/B of the long-row launch forms on
# the skewed stand-in, a short headline bench line, and a kernel trace of one
# CG + GAMG solve (tools/trace_gaps.py: busy fraction and launch gaps).
# Every GPU step has its own time limit; steps are chained so the first
# failure ends the call (no retries).
#   usage: tools/gpu_survey.sh TAG
set -o pipefail
TAG=${1:-survey}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
    || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
bash tools/gpu_gamg_setup.sh "$TAG/gamg" || exit 1
timeout -k 10 300 python -u tools/tune.py --variants bf --rounds 5 > "$OUT/bf_poisson.jsonl" 2>&1 \
    && echo "bf poisson ok" && grep -h "bitwise\|us_median" "$OUT/bf_poisson.jsonl" | tail -7 || exit 1
timeout -k 10 300 python -u tools/tune.py --matrix skewed --variants bf --rounds 3 > "$OUT/bf_skewed.jsonl" 2>&1 \
    && echo "bf skewed ok" && grep -h "bitwise\|us_median" "$OUT/bf_skewed.jsonl" | tail -7 || exit 1
timeout -k 10 300 python -u tools/tune.py --matrix fem_hex --variants bfauto --rounds 3 > "$OUT/bf_fem.jsonl" 2>&1 \
    && echo "bf fem ok" && grep -h "bitwise\|us_median" "$OUT/bf_fem.jsonl" | tail -7 || exit 1
timeout -k 10 300 python -u tools/tune.py --matrix skewed --variants overlap --rounds 5 > "$OUT/overlap.jsonl" 2>&1 \
    && echo "overlap ok" && grep us_median "$OUT/overlap.jsonl" | tail -6 || exit 1
timeout -k 10 300 python -u bench.py --no-cg --no-gamg --no-host-vec --no-flan --no-cpu-baseline --steps 100 \
    > "$OUT/head.json" 2> "$OUT/head.err" && echo "head ok" || { tail -20 "$OUT/head.err"; exit 1; }
for r in 1 2; do
  timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_graph_$r.log" 2>&1 || exit 1
  AIJHIP_KSP_NO_GRAPH=1 timeout -k 10 200 python -u tools/prof_case.py gamg > "$OUT/gamg_nograph_$r.log" 2>&1 || exit 1
  timeout -k 10 120 python -u tools/prof_case.py jacobi --its 400 > "$OUT/jac_graph_$r.log" 2>&1 || exit 1
  AIJHIP_KSP_NO_GRAPH=1 timeout -k 10 120 python -u tools/prof_case.py jacobi --its 400 > "$OUT/jac_nograph_$r.log" 2>&1 || exit 1
done
grep -H "gamg: set-up\|jacobi:" "$OUT"/gamg_*graph_*.log "$OUT"/jac_*graph_*.log
AIJHIP_KSP_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace_gamg" -o run --output-format csv \
    -- python3 tools/prof_case.py gamg > "$OUT/trace_gamg.log" 2>&1 && echo "trace ok" \
    && python3 tools/trace_gaps.py "$OUT/trace_gamg" --last 1500 | head -30
