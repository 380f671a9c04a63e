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
        s3 = line["strong_300"]  # (round 2's lines: roofline_frac; from round 3: csr_effective_frac)
        assert s3["unit"] == "GB/s" and 0 < s3.get("csr_effective_frac", s3.get("roofline_frac", 0)) < 2
    if "worst_rank" in d:  # written by distributed_block (round 2 onwards)
        assert d["worst_rank"] in [r["rank"] for r in d["ranks"]]
