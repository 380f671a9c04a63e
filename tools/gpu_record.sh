#!/bin/bash
# One GPU-box record: the -m gpu suite, smoke(), the default bench line, a
# two-rank self-launched rehearsal line (--gpus 2 --rehearse-one-gpu, both
# halo forms), and rocprofv3 kernel statistics of the headline alone and of
# the whole bench. Every GPU step has its own time limit; steps are chained so
# the first failure ends the call (no retries).
#   usage: tools/gpu_record.sh TAG [--no-tests] [--no-full-prof] [--n8]
# --n8: also the eight-rank rehearsal of the driver's N = 8 run on this one
# GPU (--gpus 8 --rehearse-one-gpu: the self-launcher's 8 children, the
# 38/37-plane 300^3 strong split (the headline), both halo forms, the distributed CG and
# CG + GAMG legs) with a weak block of 100^3 per rank.
set -o pipefail
TAG=${1:-record}; shift
TESTS=1; FULLPROF=1; N8=0
for a in "$@"; do
  case $a in --no-tests) TESTS=0 ;; --no-full-prof) FULLPROF=0 ;; --n8) N8=1 ;; esac
done
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
export TMPDIR=/tmp
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
if [ $TESTS = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
      > "$OUT/pytest.log" 2>&1 && echo "pytest ok: $(tail -1 "$OUT/pytest.log")" \
      || { grep -E "FAIL|Error" "$OUT/pytest.log" | tail -20; tail -5 "$OUT/pytest.log"; exit 1; }
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
      && tail -1 "$OUT/smoke.log" || { tail -20 "$OUT/smoke.log"; exit 1; }
fi
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
echo "bench ok"
timeout -k 10 600 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --no-gamg \
    > "$OUT/bench_rehearse_n2.json" 2> "$OUT/bench_rehearse_n2.err" \
    && echo "rehearsal n2 ok" || { tail -20 "$OUT/bench_rehearse_n2.err"; exit 1; }
if [ $N8 = 1 ]; then
  timeout -k 10 900 python -u bench.py --gpus 8 --rehearse-one-gpu --weak-grid 100 --steps 20 \
      --warmup 3 > "$OUT/bench_rehearse_n8.json" 2> "$OUT/bench_rehearse_n8.err" \
      && echo "rehearsal n8 ok" || { tail -20 "$OUT/bench_rehearse_n8.err"; exit 1; }
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_headline" -o run --output-format csv \
    -- python3 bench.py --no-cg --no-gamg --no-host-vec --no-flan --no-cpu-baseline > "$OUT/bench_headline_prof.json" \
    2> "$OUT/bench_headline_prof.err" && echo "headline prof ok" || { tail -20 "$OUT/bench_headline_prof.err"; exit 1; }
if [ $FULLPROF = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline --no-host-vec > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
      && echo "full prof ok" || { tail -20 "$OUT/bench_prof.err"; exit 1; }
fi
