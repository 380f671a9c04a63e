"""bench.py host logic (no GPU): the weak-scaling grid keeps G^3 rows per
rank in whole z-planes and reaches BASELINE configs[3]'s 600^3 at N = 8."""
import importlib.util
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 6, 8, 16])
def test_weak_grid_rows_per_rank(bench, world):
    nx, ny, nz = bench.weak_grid(300, world)
    assert nz % world == 0
    assert nx * ny * (nz // world) == 300 ** 3


def test_weak_grid_configs3(bench):
    assert bench.weak_grid(300, 1) == (300, 300, 300)
    assert bench.weak_grid(300, 2) == (300, 300, 600)
    assert bench.weak_grid(300, 4) == (300, 600, 600)
    assert bench.weak_grid(300, 8) == (600, 600, 600)


def test_weak_grid_fallback(bench):
    # 7^3 per rank cannot be split into whole planes after doubling x and y
    assert bench.weak_grid(7, 4) == (7, 7, 28)


def test_distributed_block_schema(bench):
    """The N > 1 line's `distributed` object carries world size, backend,
    RCCL version, the timeout and per rank the device and the halo-hidden
    evidence (make the 8-GPU SCALE line self-evidencing)."""
    ranks = [bench.rank_record(r, r, 0x10 + r, 27_000_000, 188_730_000, 720_000 if 0 < r < 7 else 360_000,
                               0.470 + 0.001 * r, 0.462) for r in range(8)]
    d = bench.distributed_block(8, "nccl", {"kind": "rccl", "version": 22606, "nranks": 8, "rank": 0}, 600.0, ranks)
    assert d["world_size"] == 8 and d["backend"] == "nccl" and d["comm"] == "rccl"
    assert d["rccl_version"] == 22606 and d["comm_timeout_s"] == 600.0
    assert d["worst_rank"] == 7
    for r, rec in enumerate(d["ranks"]):
        assert set(rec) == {"rank", "device", "pci_bus", "rows", "nnz", "ghosts", "spmv_us_mean",
                            "diag_block_us_mean", "halo_exposed_us"}
        assert rec["device"] == r
        assert rec["halo_exposed_us"] == round(rec["spmv_us_mean"] - rec["diag_block_us_mean"], 2)
    assert bench.distributed_block(1, "gloo", {"kind": "host", "version": 0}, 60.0, [])["rccl_version"] is None


def test_rank_record_paired_median(bench):
    """halo_forms' interleaved timing: halo_exposed_us is the median of the
    per-round differences, not the difference of two separately timed means."""
    paired = {"spmv_us_median": 470.5, "diag_us_median": 468.0, "diff_us_median": 1.25, "diff_us_iqr": [0.5, 2.0],
              "rounds": 200}
    rec = bench.rank_record(0, 0, 0x10, 27_000_000, 188_460_000, 0, 0.4810, 0.4690, paired)
    assert rec["halo_exposed_us"] == 1.25 and rec["rounds"] == 200
    assert rec["spmv_us_median"] == 470.5 and rec["diag_block_us_median"] == 468.0
    assert rec["halo_exposed_iqr_us"] == [0.5, 2.0]
    assert rec["spmv_us_mean"] == 481.0 and rec["diag_block_us_mean"] == 469.0


def test_slab_bounds_strong_300_at_8(bench):
    """The driver's N = 8 strong line splits 300 planes 38 x 4 + 37 x 4
    (DMDA PETSC_DECIDE: the first 300 % 8 ranks take one more)."""
    import importlib
    mp_mod = importlib.import_module("petsc-openacc_amd.mpiaij")
    b = [mp_mod.slab_bounds(300, 8, r) for r in range(8)]
    assert [e - s for s, e in b] == [38, 38, 38, 38, 37, 37, 37, 37]
    assert b[0][0] == 0 and b[-1][1] == 300 and all(b[i][1] == b[i + 1][0] for i in range(7))


@pytest.mark.parametrize("name", ["bench_rehearse_n2_r02e.json", "bench_mpi_n1_r02e.json",
                                  "bench_rehearse_n2_r02j.json", "bench_mpi_n1_r02j.json",
                                  "bench_rehearse_n2_r02n.json", "bench_mpi_n1_r02n.json"])
def test_committed_rehearsal_lines_carry_the_n_gt_1_fields(name):
    """The rehearsals committed under profiles/r02/ were produced by this
    bench.py: one JSON line with the contract fields plus the distributed
    block, strong_300 (N > 1) and the distributed CG / CG+GAMG."""
    import json
    line = json.loads((ROOT / "profiles" / "r02" / name).read_text().strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in line
    d = line["distributed"]
    assert d["world_size"] == line["n_gpus"] and len(d["ranks"]) == line["n_gpus"]
    assert all("halo_exposed_us" in r and "device" in r for r in d["ranks"])
    assert line["cg"]["solver"] == "aijhip_kspmpi (native)" and "host_syncs" in line["cg"]
    assert line["cg_gamg"]["its"] > 0
    if line["n_gpus"] > 1:
        s3 = line["strong_300"]  # (round 2's lines: roofline_frac; from round 4: frac)
        assert s3["unit"] == "GB/s" and 0 < s3.get("frac", s3.get("roofline_frac", 0)) <= 1
    assert_fracs_at_most_one(line)
    if "worst_rank" in d:  # written by distributed_block (round 2 onwards)
        assert d["worst_rank"] in [r["rank"] for r in d["ranks"]]


def _fracs(o, path=""):
    if isinstance(o, dict):
        for k, v in o.items():
            if "frac" in k and isinstance(v, (int, float)) and not isinstance(v, bool):
                yield f"{path}/{k}", v
            yield from _fracs(v, f"{path}/{k}")
    elif isinstance(o, list):
        for i, v in enumerate(o):
            yield from _fracs(v, f"{path}[{i}]")


def assert_fracs_at_most_one(line):
    """Every fraction of 8 TB/s a bench line reports is the bytes the timed
    kernel moves over its time: none can exceed 1."""
    bad = [(p, v) for p, v in _fracs(line) if v > 1.0]
    assert not bad, bad


def test_fraction_check_catches_an_effective_rate():
    assert_fracs_at_most_one({"roofline": {"frac": 0.74, "aj_layout": {"frac": 0.73}}, "flan": [{"frac": 0.6}]})
    with pytest.raises(AssertionError):
        assert_fracs_at_most_one({"roofline": {"csr_effective": {"frac": 1.02}}})


def test_round4_lines_have_no_fraction_above_one():
    """Lines this round's bench.py wrote (profiles/r04/bench_*.json) carry
    only fractions of the bytes each timed kernel moves."""
    import json
    for f in sorted((ROOT / "profiles" / "r04").glob("bench_*.json")):
        for raw in f.read_text().strip().splitlines():
            if raw.startswith("{"):
                assert_fracs_at_most_one(json.loads(raw))


@pytest.mark.parametrize("rec", ["af", "al", "ao", "av", "ax"])
def test_round5_records_keep_the_contract(rec):
    """Round 5's closing records (the driver's command on a GPU box): one JSON
    line with the contract's keys, a roofline with traffic counted in the run,
    a CPU baseline, every fraction <= 1, the default GAMG hierarchy PETSc's
    (53 iterations) beside the greedy one."""
    import json
    lines = [x for x in (ROOT / "profiles" / "r05" / rec / "bench.json").read_text().splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["dtype"] == "f64" and d["config"]["workload"].startswith("300^3")
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["traffic"] and r["traffic_source"].startswith("this run")
    assert d["cpu_baseline"]["kind"] == "port" and d["cpu_baseline"]["cores"] == 1
    g = d["cg_gamg"]
    assert g["its"] == 53 and g["greedy_hierarchy"]["its"] == 57
    assert_fracs_at_most_one(d)


def test_rank_plan_env_contract(bench):
    """`python bench.py --gpus N` without a launcher starts N ranks with the
    torch.distributed.run environment."""
    plan = bench.rank_plan(4, ["--gpus", "4", "--steps", "5"], 29511, env={"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert len(plan) == 4
    for r, (cmd, env) in enumerate(plan):
        assert cmd[-4:] == ["--gpus", "4", "--steps", "5"] and cmd[-5].endswith("bench.py")
        assert env["RANK"] == env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29511"
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["PATH"] == "/bin"


CHILD = ("import json, os, sys\n"
         "r = int(os.environ['RANK'])\n"
         "print('rank', r, 'noise')\n"
         "if r == int(os.environ.get('FAIL_RANK', '-1')): sys.exit(3)\n"
         "if r == 0: print(json.dumps({'n_gpus': int(os.environ['WORLD_SIZE']), 'rank': r}))\n")


def test_launch_ranks_prints_exactly_one_json_line(bench, capfd):
    import json
    import sys
    rc = bench.launch_ranks(3, [], child=[sys.executable, "-c", CHILD])
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    lines = [json.loads(x) for x in out if x.startswith("{")]
    assert lines == [{"n_gpus": 3, "rank": 0}]
    assert out == ["rank 0 noise", '{"n_gpus": 3, "rank": 0}']  # the other ranks' stdout went to stderr


def test_launch_ranks_propagates_a_failure(bench, monkeypatch):
    import sys
    monkeypatch.setenv("FAIL_RANK", "1")
    assert bench.launch_ranks(2, [], child=[sys.executable, "-c", CHILD]) == 3


def _fake_rocprof(tmp_path, body):
    exe = tmp_path / "rocprofv3"
    exe.write_text("#!/usr/bin/env python3\n" + body)
    exe.chmod(0o755)
    return exe


_FAKE_OK = r'''
import sys, pathlib
a = sys.argv
d = pathlib.Path(a[a.index("-d") + 1]); c = a[a.index("--pmc") + 1]
d.mkdir(parents=True, exist_ok=True)
v = {"FETCH_SIZE": 1000.0, "WRITE_SIZE": 300.0}[c]
k = "void aijhip::(anonymous namespace)::k_spmv_stream<512, 4094, 1, false, 0, aijhip::(anonymous namespace)::OpMult<false> >(int)"
with open(d / "run_counter_collection.csv", "w") as f:
    f.write("Kernel_Name,Counter_Name,Counter_Value\n")
    for i in range(10):
        f.write('"%s",%s,%s\n' % (k, c, v + i))
    f.write('"other_kernel(int)",%s,1e9\n' % c)
'''


def test_live_pmc_traffic_parses_the_passes(bench, tmp_path, monkeypatch):
    """roofline.traffic from two --pmc passes: 2 x FETCH_SIZE KiB + WRITE_SIZE
    KiB (MI355X_MICROARCH's gfx950 correction), mean over the headline
    kernel's dispatches, other kernels ignored (a stand-in rocprofv3)."""
    _fake_rocprof(tmp_path, _FAKE_OK)
    monkeypatch.setenv("PATH", f"{tmp_path}:{__import__('os').environ['PATH']}")
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    traffic, detail = bench.live_pmc_traffic(300, timeout_s=60)
    assert detail["read_bytes"] == int(2 * 1004.5 * 1024) and detail["write_bytes"] == int(304.5 * 1024)
    assert traffic == detail["read_bytes"] + detail["write_bytes"] and detail["dispatches"] == [10, 10]


def test_live_pmc_traffic_kills_a_hung_pass(bench, tmp_path, monkeypatch):
    """A pass that hangs (rocprofv3's 'error code 38' behaviour) is killed with
    its process group at the limit, and the bench falls back (None, reason)."""
    _fake_rocprof(tmp_path, "import time\ntime.sleep(120)\n")
    monkeypatch.setenv("PATH", f"{tmp_path}:{__import__('os').environ['PATH']}")
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    import time
    t0 = time.time()
    traffic, why = bench.live_pmc_traffic(300, timeout_s=2)
    assert traffic is None and "killed" in why and time.time() - t0 < 30


def test_live_pmc_traffic_failed_pass(bench, tmp_path, monkeypatch):
    _fake_rocprof(tmp_path, "import sys\nsys.exit(3)\n")
    monkeypatch.setenv("PATH", f"{tmp_path}:{__import__('os').environ['PATH']}")
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    traffic, why = bench.live_pmc_traffic(300, timeout_s=30)
    assert traffic is None and "exited 3" in why


def test_headline_line_n8_is_the_300_cubed_operand(bench):
    """at N > 1 `value` is the metric's 300^3 MatMult
    strong-scaled over the N GPUs (the reference's sweep), not a weak-scaled
    larger grid: 27,000,000 rows, 188,460,000 entries, SURVEY §8d's bytes."""
    info = {"kernel": "stream", "stream_threads": 512, "stream_nnz_cap": 4094, "stream_rows": 512, "nt_loads": 0,
            "column_codes": 0, "row_patterns": 0, "gather_sorted": 0}
    line = bench.headline_line(world=8, dims=(300, 300, 300), nnz_global=188_460_000, K=20, warmup=5,
                               elapsed_s=20 * 70e-6, launch_us=[70.0] * 20, layout_bytes=350_190_000, info=info,
                               distributed=True, halo="p2p", x_kind="uniform", planes=38)
    c = line["config"]
    assert c["rows"] == 27_000_000 and c["nnz"] == 188_460_000 and c["bytes_per_spmv"] == 2_801_520_004
    assert c["workload"].startswith("300^3") and "over 8 GPUs" in c["workload"]
    assert line["scaling"] == "strong" and line["n_gpus"] == 8
    assert abs(line["value"] - 2_801_520_004 / 70e-6 / 1e9) < 0.01
    assert abs(line["roofline"]["achieved"] - 350_190_000 / 70e-6 / 1e9) < 0.1
    one = bench.headline_line(world=1, dims=(300, 300, 300), nnz_global=188_460_000, K=20, warmup=5,
                              elapsed_s=20 * 480e-6, launch_us=[478.0] * 20, layout_bytes=2_801_520_004, info=info,
                              distributed=False, halo="p2p", x_kind="uniform")
    assert one["config"]["workload"].startswith("300^3 Poisson CSR MatMult_SeqAIJ (BASELINE configs[1])")
    assert one["config"]["halo"] is None and one["scaling"] == "strong"
    assert_fracs_at_most_one(line)
    assert_fracs_at_most_one(one)


def test_legs_skip_what_cannot_fit(bench):
    """A leg starts only with its budget left (else {"error": "budget"}, the
    function never called); a leg that ran is logged with its time."""
    import os
    calls = []
    legs = bench.Legs(5.0, 0, 1, False, None, lambda m: None, os.dup(1))
    legs.out = {}
    r = legs.run("gamg", 60, lambda: calls.append(1))
    assert r["error"] == "budget" and not calls and legs.out["gamg"] is r
    assert legs.log["gamg"]["status"] == "skipped"
    r = legs.run("cg", 1, lambda: {"iters": 3})
    assert r == {"iters": 3} and legs.log["cg"]["status"] == "ok"
    r = legs.run("bad", 1, lambda: 1 / 0)
    assert r["error"].startswith("ZeroDivisionError")
    s = legs.summary()
    assert s["wall_budget_s"] == 5.0 and set(s["legs"]) == {"gamg", "cg", "bad"}


WATCHDOG_CHILD = r'''
import importlib.util, sys, time
spec = importlib.util.spec_from_file_location("bench_mod", sys.argv[1])
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
legs = b.Legs(1.0, 0, 1, False, None, lambda m: print(m, file=sys.stderr), 1)
legs.out = {"metric": b.METRIC, "value": 5000.0, "cg": {"iters": 200}}
legs.headline_done = True
legs.arm()
legs.current = "cg_gamg"
time.sleep(30)
print("not reached")
'''


def test_watchdog_prints_the_line_and_exits(bench):
    """A leg still running at the deadline: rank 0 writes the line so far with
    that leg as {"error": "budget"} and the process exits 0 (the headline was
    measured) well before the leg would have finished."""
    import json
    import subprocess
    import sys
    import time
    t0 = time.time()
    p = subprocess.run([sys.executable, "-c", WATCHDOG_CHILD, str(ROOT / "bench.py")], capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 0 and time.time() - t0 < 25
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and "not reached" not in p.stdout
    d = lines[0]
    assert d["value"] == 5000.0 and d["cg"] == {"iters": 200}
    assert d["cg_gamg"]["error"] == "budget" and d["budget"]["legs"]["cg_gamg"]["status"] == "cut at the deadline"


@pytest.mark.parametrize("rec,world", [("a/bench_mpi_n1_gamgdist.json", 1), ("e/bench_rehearse_n2.json", 2),
                                       ("k/bench_rehearse_n8.json", 8)])
def test_round6_distributed_records_measure_the_metric(rec, world):
    """VERDICT r05 item 1, on the records this bench.py wrote on a GPU box
    (profiles/r06/): the distributed line's `value` is the 300^3 operand
    itself (27,000,000 rows, 188,460,000 entries) strong-scaled over the
    ranks, the CPU baselines (1 core and all cores) are present at every N,
    the weak block beside it at N > 1, every leg within the wall budget's
    bookkeeping, and the distributed CG + GAMG at the full per-rank size
    takes the single-GPU hierarchy's 53 iterations (PETSc's parallel MIS,
    partition-independent)."""
    import json
    lines = [x for x in (ROOT / "profiles" / "r06" / rec).read_text().splitlines() if x.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["scaling"] == "strong"
    c = d["config"]
    assert c["rows"] == 27_000_000 and c["nnz"] == 188_460_000 and c["workload"].startswith("300^3")
    assert d["cpu_baseline"]["cores"] == 1 and d["cpu_baseline"]["kind"] == "port"
    assert d["cpu_baseline_all_cores"]["cores"] >= 1 and d["cpu_baseline_all_cores"]["value"] > 0
    assert abs(d["value"] - c["bytes_per_spmv"] * d["steps"] / (d["ms_per_step"] * d["steps"] / 1e3) / 1e9) \
        < 0.01 * d["value"]
    if world > 1:
        assert d["weak"]["scaling"] == "weak" and "error" not in d["weak"]
    g = d["cg_gamg"]
    assert g["its"] == 53 and [lv["rows"] for lv in g["levels"]][:3] == [27_000_000, 2_413_301, 183_694]
    assert set(d["budget"]["legs"]) >= {"cg", "cg_gamg", "cpu_baseline"}
    assert_fracs_at_most_one(d)
