# Row-template x window A/B (AIJHIP_TMPL_WINDOW=1 default / 0 gathering):
# the template GPU tests, then the bench's effective, CG and CG + GAMG legs
# in alternating processes.   bash tools/runs/win_ab.sh TAG [WINDOW ...]
set -o pipefail
OUT=gpurun_out/r06/${1:?tag}; shift; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_row_patterns_gpu.py -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
i=0
for w in "${@:-1 0 1 0}"; do
  i=$((i + 1))
  AIJHIP_TMPL_WINDOW=$w timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-host-vec --no-flan --no-pmc \
    --no-cpu-baseline > $OUT/bench_${i}_w$w.json 2> $OUT/bench_${i}_w$w.err || { tail -20 $OUT/bench_${i}_w$w.err; exit 1; }
  python3 - $OUT/bench_${i}_w$w.json $w <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e, c, g = d.get("effective") or {}, d.get("cg") or {}, d.get("cg_gamg") or {}
print("window", sys.argv[2], "effective us", e.get("us_mean"), "cg it/s", c.get("iters_per_s"),
      "gamg its", g.get("its"), "solve s", g.get("solve_s"))
EOF
done
