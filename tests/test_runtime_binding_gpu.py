"""The library and PyTorch share one HIP runtime whatever the import order.

PyTorch's wheel carries its own libamdhip64 under the same soname as
/opt/rocm's. A process that loaded libaijhip.so before importing torch used
to hold two runtimes, and the one initialised second saw no device. Each
case runs in a fresh interpreter (load order is per process)."""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent

SCRIPT = r"""
import ctypes, importlib, re, sys
sys.path.insert(0, {root!r})
pkg = importlib.import_module("petsc-openacc_amd")
order = {order!r}

def count():
    c = ctypes.c_int(0)
    rc = pkg.lib().aijhip_device_count(ctypes.byref(c))
    return rc, c.value

if order == "lib_first":
    pkg.poisson_csr(4)                     # loads libaijhip.so before torch
    import torch
    assert torch.cuda.is_available()       # torch initialises first
    rc, n = count()
    assert rc == 0 and n >= 1, (rc, n, pkg.lib().aijhip_last_error())
else:
    rc, n = count()                        # the library initialises first
    assert rc == 0 and n >= 1, (rc, n)
    import torch
    assert torch.cuda.is_available()
    assert torch.ones(3, device="cuda").sum().item() == 3.0
runtimes = set(re.findall(r"\S*libamdhip64\S*", open("/proc/self/maps").read()))
assert len(runtimes) == 1, runtimes
with pkg.SeqAIJHIP(*pkg.poisson_csr(4)) as A:
    x = torch.ones(64, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    A.mult(x, y)
    torch.cuda.synchronize()
print("ok", order, sorted(runtimes))
"""


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["lib_first", "lib_initialises_first"])
def test_gpu_library_and_torch_share_one_hip_runtime(order):
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=str(ROOT), order=order)], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout
