"""petsc-openacc_amd — MI355X-native sequential-AIJ SpMV for PETSc's KSP hot path.

Host-side mirror of the operator interface the reference patches
(MatMult_SeqAIJ / MatAssemblyEnd_SeqAIJ / MatDestroy_SeqAIJ, see
include/aijhip.h for the file:line map) over the C ABI in lib/libaijhip.so.
PyTorch is used only for device memory and streams: vectors are float64 CUDA
(HIP) tensors whose pointers go straight to the C ABI.

There is no CPU fallback: if libaijhip.so is missing or no gfx950 device is
visible, every compute call raises AIJHIPError.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

_PKG = Path(__file__).resolve().parent
LIB_PATH = _PKG / "lib" / "libaijhip.so"
# A/B timing of two builds in alternating processes (tools/build_ab.sh) may
# name another build of the same library, but only with AIJHIP_AB=1 set too,
# and the process says so on stderr: nothing loads a foreign build silently.
if os.environ.get("AIJHIP_LIB"):
    if os.environ.get("AIJHIP_AB") != "1":
        raise RuntimeError("AIJHIP_LIB is set without AIJHIP_AB=1: refusing to load a build other than "
                           f"{LIB_PATH}")
    LIB_PATH = Path(os.environ["AIJHIP_LIB"]).resolve()
    import sys as _sys
    print(f"[aijhip] A/B run: loading {LIB_PATH}", file=_sys.stderr)

KERNELS = {"auto": 0, "stream": 1, "scalar": 2, "vector": 3, "merge": 4}
KERNEL_NAMES = {v: k for k, v in KERNELS.items()}
OPTIONS = {"geometry": 1, "nt_loads": 3, "exact": 6, "long_xcd": 8, "long_overlap": 9, "host_pipeline": 10,
           "gather_sort": 12, "column_codes": 13, "row_patterns": 14, "row_templates": 17,
           "value_codes": 18}
# withdrawn in ABI 2 (measured slower, profiles/README.md "Measured and withdrawn"); the library refuses them
WITHDRAWN_OPTIONS = {"xcd_remap": 2, "persistent": 4, "clamped": 5, "x_tile": 7, "row_group": 11,
                     "long_window": 15, "pipeline": 16}

AIJHIP_OK, AIJHIP_ERR_ARG, AIJHIP_ERR_ALLOC, AIJHIP_ERR_HIP, AIJHIP_ERR_NODEVICE, AIJHIP_ERR_STATE = range(6)

# Every symbol include/aijhip.h and include/aijhip_harness.h declare.
ABI_SYMBOLS = (
    "aijhip_abi_version", "aijhip_last_error", "aijhip_device_count",
    "aijhip_mat_create", "aijhip_mat_create_from_device", "aijhip_mat_set_kernel", "aijhip_mat_set_option",
    "aijhip_mat_update_values", "aijhip_mat_assembly_end", "aijhip_mat_mult",
    "aijhip_mat_mult_add", "aijhip_mat_mult_transpose", "aijhip_mat_mult_host",
    "aijhip_mat_mult_add_host", "aijhip_mat_mult_transpose_host",
    "aijhip_mat_get_info", "aijhip_mat_get_device_csr", "aijhip_mat_destroy",
)
HARNESS_SYMBOLS = (
    "aijhip_poisson_nnz", "aijhip_poisson_fill", "aijhip_poisson_vectors",
    "aijhip_splitmix_uniform", "aijhip_skewed_csr", "aijhip_fem_hex_csr", "aijhip_split_rows",
    "aijhip_poisson_fill_device", "aijhip_poisson_vectors_device", "aijhip_mat_create_poisson",
)


class AIJHIPError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"aijhip error {code}: {msg}")
        self.code = code


class AIJInfo(ctypes.Structure):
    _fields_ = [
        ("m", ctypes.c_int32), ("n", ctypes.c_int32), ("nz", ctypes.c_int64),
        ("nonzerorowcnt", ctypes.c_int32), ("max_row_nz", ctypes.c_int32),
        ("compressed_row", ctypes.c_int32), ("kernel", ctypes.c_int32),
        ("vector_lanes", ctypes.c_int32), ("n_blocks", ctypes.c_int32),
        ("n_long_rows", ctypes.c_int32), ("device", ctypes.c_int32),
        ("device_bytes", ctypes.c_int64), ("mult_flops", ctypes.c_double),
        ("mult_bytes", ctypes.c_int64),
        ("stream_geometry", ctypes.c_int32), ("nt_loads", ctypes.c_int32),
        ("stream_threads", ctypes.c_int32), ("stream_nnz_cap", ctypes.c_int32), ("stream_rows", ctypes.c_int32),
        ("exact", ctypes.c_int32), ("gather_sorted", ctypes.c_int32), ("column_codes", ctypes.c_int32),
        ("row_patterns", ctypes.c_int32),
        ("long_overlap", ctypes.c_int32),
        ("mult_layout_bytes", ctypes.c_int64),
        ("hw_queues", ctypes.c_int32), ("row_templates", ctypes.c_int32), ("value_codes", ctypes.c_int32),
        ("reserved1", ctypes.c_int32),
    ]


_lib = None
_P = ctypes.c_void_p
_I32P = ctypes.POINTER(ctypes.c_int32)
_I64P = ctypes.POINTER(ctypes.c_int64)
_F64P = ctypes.POINTER(ctypes.c_double)


def _bind_process_hip_runtime() -> None:
    """One HIP runtime per process. PyTorch ships its own libamdhip64 under
    the same soname (libamdhip64.so.7) as /opt/rocm's and loads it by path. If
    this library came first it would bind ROCm's copy, torch would then load
    its own, and whichever of the two initialised second would find no device
    ("no ROCm-capable device is detected"; tests/test_runtime_binding_gpu.py).
    Loading torch's copy first (without importing torch) makes the soname
    resolve to it for both."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    hip = Path(spec.origin).parent / "lib" / "libamdhip64.so"
    if hip.exists():
        ctypes.CDLL(str(hip), mode=ctypes.RTLD_GLOBAL)


def lib() -> ctypes.CDLL:
    """Load lib/libaijhip.so (built by build.py); fail loudly if absent."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise AIJHIPError(AIJHIP_ERR_STATE, f"{LIB_PATH} is missing — run petsc-openacc_amd/build.py "
                                                "(there is no CPU fallback)")
        _bind_process_hip_runtime()
        L = ctypes.CDLL(str(LIB_PATH))
        L.aijhip_last_error.restype = ctypes.c_char_p
        for name in ABI_SYMBOLS + HARNESS_SYMBOLS:
            f = getattr(L, name)
            if name not in ("aijhip_last_error", "aijhip_splitmix_uniform"):
                f.restype = ctypes.c_int
        L.aijhip_splitmix_uniform.restype = None
        L.aijhip_mat_create.argtypes = [ctypes.c_int, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                        _P, _P, _P, ctypes.POINTER(_P)]
        L.aijhip_mat_create_from_device.argtypes = L.aijhip_mat_create.argtypes
        L.aijhip_mat_set_kernel.argtypes = [_P, ctypes.c_int, ctypes.c_int]
        L.aijhip_mat_set_option.argtypes = [_P, ctypes.c_int, ctypes.c_int]
        L.aijhip_mat_update_values.argtypes = [_P, _P]
        L.aijhip_mat_assembly_end.argtypes = [_P, ctypes.c_int64, _P, _P, _P]
        L.aijhip_mat_mult.argtypes = [_P, _P, _P, _P]
        L.aijhip_mat_mult_add.argtypes = [_P, _P, _P, _P, _P]
        L.aijhip_mat_mult_transpose.argtypes = [_P, _P, _P, _P]
        L.aijhip_mat_mult_host.argtypes = [_P, _P, _P]
        L.aijhip_mat_mult_add_host.argtypes = [_P, _P, _P, _P]
        L.aijhip_mat_mult_transpose_host.argtypes = [_P, _P, _P]
        L.aijhip_mat_get_info.argtypes = [_P, ctypes.POINTER(AIJInfo)]
        L.aijhip_mat_get_device_csr.argtypes = [_P, ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P)]
        L.aijhip_mat_destroy.argtypes = [_P]
        L.aijhip_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.aijhip_poisson_nnz.argtypes = [ctypes.c_int32] * 5 + [_I64P]
        L.aijhip_poisson_fill.argtypes = [ctypes.c_int32] * 5 + [ctypes.c_int, _P, _P, _P, _F64P]
        L.aijhip_poisson_vectors.argtypes = [ctypes.c_int32] * 5 + [ctypes.c_int, _P, _P]
        L.aijhip_splitmix_uniform.argtypes = [ctypes.c_int64, ctypes.c_uint64, ctypes.c_int64, _P]
        L.aijhip_skewed_csr.argtypes = [ctypes.c_int32, ctypes.c_uint64, _I64P, _P, _P, _P]
        L.aijhip_fem_hex_csr.argtypes = [ctypes.c_int32] * 4 + [ctypes.c_uint64, _I64P, _P, _P, _P]
        L.aijhip_poisson_fill_device.argtypes = [ctypes.c_int32] * 5 + [ctypes.c_int, _P, _P, _P, _F64P, _P]
        L.aijhip_poisson_vectors_device.argtypes = [ctypes.c_int32] * 5 + [ctypes.c_int, _P, _P, _P]
        L.aijhip_mat_create_poisson.argtypes = [ctypes.c_int] + [ctypes.c_int32] * 5 + [ctypes.c_int, _F64P,
                                                                                         ctypes.POINTER(_P)]
        L.aijhip_split_rows.argtypes = [ctypes.c_int32, _P, _P, _P, ctypes.c_int32, ctypes.c_int32,
                                        _I64P, _I64P, _I32P, _P, _P, _P, _P, _P, _P, _P]
        _lib = L
    return _lib


def _check(rc: int):
    if rc != AIJHIP_OK:
        raise AIJHIPError(rc, lib().aijhip_last_error().decode(errors="replace"))


def _np_ptr(a: np.ndarray, dtype) -> int:
    if a.dtype != dtype or not a.flags["C_CONTIGUOUS"]:
        raise TypeError(f"expected contiguous {np.dtype(dtype)} array, got {a.dtype}")
    return a.ctypes.data


def _dev_ptr(t, n: int, what: str) -> int:
    import torch
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{what}: expected a torch tensor on the GPU")
    if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous():
        raise TypeError(f"{what}: expected a contiguous float64 GPU tensor")
    if t.numel() < n:
        raise ValueError(f"{what}: has {t.numel()} entries, needs {n}")
    return t.data_ptr()


def _stream_handle(stream) -> int:
    import torch
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def device_count() -> int:
    c = ctypes.c_int(0)
    rc = lib().aijhip_device_count(ctypes.byref(c))
    return c.value if rc == AIJHIP_OK else 0


def poisson_device(nx: int, ny: int | None = None, nz: int | None = None, z0: int = 0, z1: int | None = None,
                   ref_point: bool = True, device: int = 0):
    """The helper.cpp operand assembled on the device (aijhip_mat_create_poisson):
    returns (SeqAIJHIP, setRefPoint scale) with no host CSR."""
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    z1 = nz if z1 is None else z1
    h = _P()
    sc = ctypes.c_double()
    _check(lib().aijhip_mat_create_poisson(device, nx, ny, nz, z0, z1, int(ref_point), ctypes.byref(sc),
                                           ctypes.byref(h)))
    return SeqAIJHIP(None, None, None, device=device, _handle=h), sc.value


def poisson_vectors_device(nx: int, ny: int | None = None, nz: int | None = None, z0: int = 0,
                           z1: int | None = None, ref_point: bool = True, rhs=None, exact=None, stream=None):
    """generateRHS / generateExt on the device into float64 GPU tensors."""
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    z1 = nz if z1 is None else z1
    mloc = (z1 - z0) * nx * ny
    _check(lib().aijhip_poisson_vectors_device(
        nx, ny, nz, z0, z1, int(ref_point), _dev_ptr(rhs, mloc, "rhs") if rhs is not None else None,
        _dev_ptr(exact, mloc, "exact") if exact is not None else None, _stream_handle(stream)))


class SeqAIJHIP:
    """A device-resident SeqAIJ matrix: the Mat the reference's patches act on.

    Construction uploads the CSR once (MatAssemblyEnd hook, step2
    MatAssemblyEnd patch:42-44); `mult` is MatMult_SeqAIJ with device-resident
    vectors; `destroy` frees the device copy (MatDestroy hook, patch:18-34).
    """

    def __init__(self, ai, aj, aa, ncols: int | None = None, device: int = 0, kernel: str = "auto",
                 lanes: int = 0, _handle=None, **options):
        if _handle is not None:  # adopt a handle made on the device (poisson_device)
            self._h = _handle
            inf = self.info()
            self.m, self.n, self.nz, self.device = inf["m"], inf["n"], inf["nz"], device
            return
        ai = np.ascontiguousarray(ai, dtype=np.int32)
        aj = np.ascontiguousarray(aj, dtype=np.int32)
        aa = np.ascontiguousarray(aa, dtype=np.float64)
        m = len(ai) - 1
        if ncols is None:
            ncols = m
        self._h = _P()
        _check(lib().aijhip_mat_create(device, m, ncols, len(aj), _np_ptr(ai, np.int32),
                                       _np_ptr(aj, np.int32), _np_ptr(aa, np.float64), ctypes.byref(self._h)))
        self.m, self.n, self.nz, self.device = m, int(ncols), int(len(aj)), device
        if kernel != "auto" or lanes:
            self.set_kernel(kernel, lanes)
        for k, v in options.items():  # speed / ordering knobs: geometry, exact, ...
            self.set_option(k, v)

    # ---- PETSc MatOps analogues
    def set_kernel(self, kernel: str, lanes: int = 0):
        _check(lib().aijhip_mat_set_kernel(self._h, KERNELS[kernel], lanes))

    def set_option(self, option: str, value: int):
        """Speed-only STREAM knobs (include/aijhip.h AIJHIP_OPT_*): geometry,
        nt_loads, exact, long_xcd, host_pipeline, gather_sort,
        column_codes, row_patterns, row_templates. Results never depend on them."""
        code = OPTIONS.get(option, WITHDRAWN_OPTIONS.get(option))
        if code is None:
            raise KeyError(f"unknown option {option!r}")
        _check(lib().aijhip_mat_set_option(self._h, code, int(value)))

    def mult(self, x, y, stream=None):
        """y = A x (MatMult_SeqAIJ). x: float64[n], y: float64[m] GPU tensors."""
        _check(lib().aijhip_mat_mult(self._h, _dev_ptr(x, self.n, "x"), _dev_ptr(y, self.m, "y"),
                                     _stream_handle(stream)))

    def mult_add(self, x, z, w, stream=None):
        """w = z + A x (MatMultAdd_SeqAIJ)."""
        _check(lib().aijhip_mat_mult_add(self._h, _dev_ptr(x, self.n, "x"), _dev_ptr(z, self.m, "z"),
                                         _dev_ptr(w, self.m, "w"), _stream_handle(stream)))

    def mult_transpose(self, x, y, stream=None):
        """y = A^T x (MatMultTranspose_SeqAIJ)."""
        _check(lib().aijhip_mat_mult_transpose(self._h, _dev_ptr(x, self.m, "x"),
                                               _dev_ptr(y, self.n, "y"), _stream_handle(stream)))

    def mult_host(self, x: np.ndarray, out: np.ndarray | None = None) -> np.ndarray:
        """Step-2 semantics: host x in, host y out (copies over PCIe,
        pipelined with the product as steps 3/4 do; pinned arrays, e.g. numpy
        views of torch pin_memory tensors, are DMA'd without staging)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        if x.shape[0] < self.n:
            raise ValueError("x too short")
        y = np.empty(self.m) if out is None else out
        if y.shape[0] < self.m:
            raise ValueError("out too short")
        _check(lib().aijhip_mat_mult_host(self._h, _np_ptr(x, np.float64), _np_ptr(y, np.float64)))
        return y

    def mult_add_host(self, x: np.ndarray, z: np.ndarray, out: np.ndarray | None = None) -> np.ndarray:
        """w = z + A x with host arrays (MatMultAdd_SeqAIJ); out may be z."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        z = np.ascontiguousarray(z, dtype=np.float64)
        if x.shape[0] < self.n or z.shape[0] < self.m:
            raise ValueError("x or z too short")
        w = np.empty(self.m) if out is None else out
        if w.shape[0] < self.m:
            raise ValueError("out too short")
        _check(lib().aijhip_mat_mult_add_host(self._h, _np_ptr(x, np.float64), _np_ptr(z, np.float64),
                                              _np_ptr(w, np.float64)))
        return w

    def mult_transpose_host(self, x: np.ndarray, out: np.ndarray | None = None) -> np.ndarray:
        """y = A^T x with host arrays (MatMultTranspose_SeqAIJ)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        if x.shape[0] < self.m:
            raise ValueError("x too short")
        y = np.empty(self.n) if out is None else out
        if y.shape[0] < self.n:
            raise ValueError("out too short")
        _check(lib().aijhip_mat_mult_transpose_host(self._h, _np_ptr(x, np.float64), _np_ptr(y, np.float64)))
        return y

    def update_values(self, aa):
        aa = np.ascontiguousarray(aa, dtype=np.float64)
        if aa.shape[0] != self.nz:
            raise ValueError("update_values: nz mismatch")
        _check(lib().aijhip_mat_update_values(self._h, _np_ptr(aa, np.float64)))

    def assembly_end(self, ai, aj, aa):
        ai = np.ascontiguousarray(ai, dtype=np.int32)
        aj = np.ascontiguousarray(aj, dtype=np.int32)
        aa = np.ascontiguousarray(aa, dtype=np.float64)
        if len(ai) - 1 != self.m:
            raise ValueError("assembly_end: row count changed")
        _check(lib().aijhip_mat_assembly_end(self._h, len(aj), _np_ptr(ai, np.int32), _np_ptr(aj, np.int32),
                                             _np_ptr(aa, np.float64)))
        self.nz = int(len(aj))

    def info(self) -> dict:
        inf = AIJInfo()
        _check(lib().aijhip_mat_get_info(self._h, ctypes.byref(inf)))
        d = {f: getattr(inf, f) for f, _ in AIJInfo._fields_}
        d["kernel"] = KERNEL_NAMES.get(d["kernel"], d["kernel"])
        return d

    def device_csr(self):
        """(ai, aj, aa) device pointers of the handle's CSR copy (borrowed)."""
        p = [_P(), _P(), _P()]
        _check(lib().aijhip_mat_get_device_csr(self._h, *[ctypes.byref(q) for q in p]))
        return tuple(q.value for q in p)

    def destroy(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().aijhip_mat_destroy(self._h)
            self._h = _P()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ----------------------------------------------------------------- operands
def poisson_csr(nx: int, ny: int | None = None, nz: int | None = None, z0: int = 0, z1: int | None = None,
                ref_point: bool = True):
    """CSR rows of the reference Poisson operand for the z-slab [z0, z1)
    (helper.cpp:161-279 restated in harness.cpp). Columns are global."""
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    z1 = nz if z1 is None else z1
    L = lib()
    nnz = ctypes.c_int64()
    _check_h(L.aijhip_poisson_nnz(nx, ny, nz, z0, z1, ctypes.byref(nnz)), "poisson_nnz")
    mloc = nx * ny * (z1 - z0)
    ai = np.empty(mloc + 1, np.int32)
    aj = np.empty(nnz.value, np.int32)
    aa = np.empty(nnz.value, np.float64)
    scale = ctypes.c_double()
    _check_h(L.aijhip_poisson_fill(nx, ny, nz, z0, z1, int(ref_point), ai.ctypes.data, aj.ctypes.data,
                                   aa.ctypes.data, ctypes.byref(scale)), "poisson_fill")
    return ai, aj, aa


def poisson_vectors(nx: int, ny: int | None = None, nz: int | None = None, z0: int = 0, z1: int | None = None,
                    ref_point: bool = True):
    """(rhs, exact) of the reference problem (helper.cpp:78-157, :250-279)."""
    ny = nx if ny is None else ny
    nz = nx if nz is None else nz
    z1 = nz if z1 is None else z1
    mloc = nx * ny * (z1 - z0)
    rhs = np.empty(mloc)
    exact = np.empty(mloc)
    _check_h(lib().aijhip_poisson_vectors(nx, ny, nz, z0, z1, int(ref_point), rhs.ctypes.data,
                                          exact.ctypes.data), "poisson_vectors")
    return rhs, exact


def splitmix_uniform(n: int, seed: int = 42, offset: int = 0) -> np.ndarray:
    x = np.empty(n)
    lib().aijhip_splitmix_uniform(n, seed, offset, x.ctypes.data)
    return x


FLAN_1565_ROWS = 1564794


def skewed_csr(m: int = FLAN_1565_ROWS, seed: int = 1565):
    """Seeded skewed CSR standing in for SuiteSparse Flan_1565 (absent offline)."""
    L = lib()
    nnz = ctypes.c_int64()
    _check_h(L.aijhip_skewed_csr(m, seed, ctypes.byref(nnz), None, None, None), "skewed_csr")
    ai = np.empty(m + 1, np.int32)
    aj = np.empty(nnz.value, np.int32)
    aa = np.empty(nnz.value, np.float64)
    _check_h(L.aijhip_skewed_csr(m, seed, ctypes.byref(nnz), ai.ctypes.data, aj.ctypes.data, aa.ctypes.data),
             "skewed_csr")
    return ai, aj, aa


FLAN_HEX_GRID = (81, 80, 80)  # 518,400 nodes x 3 dofs = 1,555,200 rows (Flan_1565: 1,564,794)


def fem_hex_csr(nx: int = FLAN_HEX_GRID[0], ny: int = FLAN_HEX_GRID[1], nz: int = FLAN_HEX_GRID[2],
                dofs: int = 3, seed: int = 1565):
    """Seeded FEM-structured CSR standing in for Flan_1565's mesh structure
    (3-D hexahedral, 3 dofs per node, 27-node coupling)."""
    L = lib()
    nnz = ctypes.c_int64()
    _check_h(L.aijhip_fem_hex_csr(nx, ny, nz, dofs, seed, ctypes.byref(nnz), None, None, None), "fem_hex_csr")
    m = nx * ny * nz * dofs
    ai = np.empty(m + 1, np.int32)
    aj = np.empty(nnz.value, np.int32)
    aa = np.empty(nnz.value, np.float64)
    _check_h(L.aijhip_fem_hex_csr(nx, ny, nz, dofs, seed, ctypes.byref(nnz), ai.ctypes.data, aj.ctypes.data,
                                  aa.ctypes.data), "fem_hex_csr")
    return ai, aj, aa


def split_rows(ai, aj, aa, col_lo: int, col_hi: int):
    """PETSc MPIAIJ split: (diag CSR, offdiag CSR, garray)."""
    ai = np.ascontiguousarray(ai, dtype=np.int32)
    aj = np.ascontiguousarray(aj, dtype=np.int32)
    aa = np.ascontiguousarray(aa, dtype=np.float64)
    m = len(ai) - 1
    L = lib()
    nzd, nzo, ng = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
    args = (m, ai.ctypes.data, aj.ctypes.data, aa.ctypes.data, col_lo, col_hi,
            ctypes.byref(nzd), ctypes.byref(nzo), ctypes.byref(ng))
    _check_h(L.aijhip_split_rows(*args, None, None, None, None, None, None, None), "split_rows")
    d_ai = np.empty(m + 1, np.int32); d_aj = np.empty(nzd.value, np.int32); d_aa = np.empty(nzd.value)
    o_ai = np.empty(m + 1, np.int32); o_aj = np.empty(nzo.value, np.int32); o_aa = np.empty(nzo.value)
    garray = np.empty(ng.value, np.int32)
    _check_h(L.aijhip_split_rows(*args, d_ai.ctypes.data, d_aj.ctypes.data, d_aa.ctypes.data,
                                 o_ai.ctypes.data, o_aj.ctypes.data, o_aa.ctypes.data, garray.ctypes.data),
             "split_rows")
    return (d_ai, d_aj, d_aa), (o_ai, o_aj, o_aa), garray


def _check_h(rc: int, what: str):
    if rc != AIJHIP_OK:
        raise AIJHIPError(rc, f"{what} failed (bad arguments)")


def algorithmic_bytes(m: int, ncols: int, nnz: int) -> int:
    """12 nnz + 4 (m+1) + 8 ncols + 8 m bytes per SpMV."""
    return 12 * nnz + 4 * (m + 1) + 8 * ncols + 8 * m
