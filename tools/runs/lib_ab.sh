# A/B of two library builds (tools/build_ab.sh): the GPU tests named in
# TESTS on the working tree's build, then the bench's effective, CG and
# CG + GAMG legs alternating between ablibs/$BASE and the working tree.
#   TESTS="tests/a.py tests/b.py" bash tools/runs/lib_ab.sh TAG BASE [ROUNDS]
set -o pipefail
OUT=gpurun_out/r06/${1:?tag}; BASE=${2:?base}; N=${3:-2}; mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread \
    > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
summ() {
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e, c, g = d.get("effective") or {}, d.get("cg") or {}, d.get("cg_gamg") or {}
print(sys.argv[2], "effective us", e.get("us_mean"), "cg it/s", c.get("iters_per_s"), "gamg its", g.get("its"),
      "solve s", g.get("solve_s"))
EOF
}
for i in $(seq 1 $N); do
  for lib in new base; do
    env=""
    [ $lib = base ] && env="AIJHIP_AB=1 AIJHIP_LIB=ablibs/$BASE/libaijhip.so"
    f=$OUT/bench_${i}_$lib
    eval "$env timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-host-vec --no-flan --no-pmc \
      --no-cpu-baseline" > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
    summ $f.json "$lib"
  done
done
