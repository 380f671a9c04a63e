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
