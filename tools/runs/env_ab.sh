# A/B of environment switches on the bench's effective, CG and CG + GAMG
# legs, alternating processes:
#   bash tools/runs/env_ab.sh TAG ROUNDS "VAR=VAL ..." "VAR=VAL ..." ...
set -o pipefail
OUT=gpurun_out/r06/${1:?tag}; N=${2:?rounds}; shift 2; mkdir -p $OUT
export TMPDIR=/tmp
for i in $(seq 1 $N); do
  k=0
  for cfg in "$@"; do
    k=$((k + 1))
    f=$OUT/bench_${i}_$k
    eval "$cfg timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-host-vec --no-flan --no-pmc \
      --no-cpu-baseline" > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
    python3 - $f.json "$cfg" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e, c, g = d.get("effective") or {}, d.get("cg") or {}, d.get("cg_gamg") or {}
print(sys.argv[2], "| effective us", e.get("us_mean"), "cg it/s", c.get("iters_per_s"), "gamg its", g.get("its"),
      "solve s", g.get("solve_s"))
EOF
  done
done
