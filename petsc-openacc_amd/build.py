"""Build the in-tree shared libraries (gfx950 only).

    python petsc-openacc_amd/build.py          # libaijhip.so (+ the oracle)

libaijhip.so  — the product: HIP kernels + C ABI (include/aijhip.h) + host
                operand producers (include/aijhip_harness.h).
oracle/liboracle.so — the CPU checker (test infrastructure only).
Both are git-ignored and travel to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
LIB = LIBDIR / "libaijhip.so"
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "liboracle.so"

HIP_SOURCES = ["aijhip_kernels.hip", "aijhip_api.cpp", "ksp.hip", "poisson.hip", "gamg_device.hip", "vec.hip",
               "ksp_mpi.hip", "host_pipe.cpp", "gamg_aggregate.hip", "gamg_mpi.hip"]
HOST_SOURCES = ["harness.cpp", "gamg_setup.cpp"]
ARCH = os.environ.get("AIJHIP_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found: the HIP path cannot be built")


def _digest(deps, extra=()) -> str:
    """sha256 over the sources (names and contents) and the compile lines."""
    import hashlib
    h = hashlib.sha256()
    for d in sorted(Path(p) for p in deps):
        h.update(d.name.encode() + b"\0" + d.read_bytes() + b"\0")
    for e in extra:
        h.update(str(e).encode() + b"\0")
    return h.hexdigest()


def _stale(target: Path, deps, extra=()) -> bool:
    """A target is stale unless the digest recorded beside it when it was built
    equals the digest of its sources now. Content, not mtime: a snapshot copied
    to another machine keeps its prebuilt library only if it was built from
    exactly these sources and flags."""
    stamp = target.with_name(target.name + ".sha256")
    if not target.exists() or not stamp.exists():
        return True
    return stamp.read_text().strip() != _digest(deps, extra)


def _stamp(target: Path, deps, extra=()) -> None:
    target.with_name(target.name + ".sha256").write_text(_digest(deps, extra) + "\n")


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: " + " ".join(map(str, cmd)) + "\n" + r.stdout + r.stderr)


def build_lib(force: bool = False) -> Path:
    LIBDIR.mkdir(exist_ok=True)
    srcs = [CSRC / s for s in HIP_SOURCES + HOST_SOURCES if (CSRC / s).exists()]
    deps = srcs + list(CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h"))
    common = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", f"-I{ROOT / 'include'}", f"-I{CSRC}"]
    flags = (ARCH, *common)
    if not force and not _stale(LIB, deps, flags):
        return LIB
    objdir = PKG / "build"
    objdir.mkdir(exist_ok=True)
    hipcc = _hipcc()
    objs, jobs = [], []
    for s in srcs:
        o = objdir / (s.stem + ".o")
        if s.name in HOST_SOURCES:
            cmd = ["g++", *common, "-fopenmp", "-c", str(s), "-o", str(o)]
        else:
            cmd = [hipcc, "-x", "hip", f"--offload-arch={ARCH}", *common, "-c", str(s), "-o", str(o)]
        odeps = [s, *CSRC.glob("*.h"), *(ROOT / "include").glob("*.h")]
        if force or _stale(o, odeps, cmd):
            jobs.append((cmd, o, odeps))
        objs.append(str(o))

    def _compile(job):
        cmd, o, odeps = job
        _run(cmd)
        _stamp(o, odeps, cmd)

    # translation units compile in parallel (at most 8 at once)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(_compile, jobs))
    tmp = LIB.with_suffix(".so.tmp")
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *objs, "-lgomp",
          "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"])
    os.replace(tmp, LIB)
    _stamp(LIB, deps, flags)
    return LIB


MAIN_KSP = PKG / "bin" / "main_ksp"


def build_main_ksp(force: bool = False) -> Path:
    """The main_ksp.cpp-equivalent driver, linked against libaijhip.so."""
    lib = build_lib(force)
    src = CSRC / "main_ksp.cpp"
    mdeps = [src, lib.with_name(lib.name + ".sha256"), *(ROOT / "include").glob("*.h")]
    if not force and not _stale(MAIN_KSP, mdeps, (ARCH,)):
        return MAIN_KSP
    MAIN_KSP.parent.mkdir(exist_ok=True)
    tmp = MAIN_KSP.with_suffix(".tmp")
    _run([_hipcc(), "-x", "hip", f"--offload-arch={ARCH}", "-O2", "-std=c++17", f"-I{ROOT / 'include'}",
          str(src), "-o", str(tmp), f"-L{LIBDIR}", "-laijhip", "-Wl,-rpath,$ORIGIN/../lib"])
    os.replace(tmp, MAIN_KSP)
    _stamp(MAIN_KSP, mdeps, (ARCH,))
    return MAIN_KSP


def build_oracle(force: bool = False) -> Path:
    srcs = [ORACLE_DIR / "matmult_seqaij.c", ORACLE_DIR / "cg_gamg.c"]
    if not force and not _stale(ORACLE_LIB, srcs):
        return ORACLE_LIB
    tmp = ORACLE_LIB.with_suffix(".so.tmp")
    # -ffp-contract=off: each product is rounded before it is added (PETSc's
    # x86 build has no FMA at -march=x86-64 either).
    _run(["gcc", "-O2", "-fPIC", "-shared", "-fopenmp", "-ffp-contract=off", "-o", str(tmp), *map(str, srcs), "-lm"])
    os.replace(tmp, ORACLE_LIB)
    _stamp(ORACLE_LIB, srcs)
    return ORACLE_LIB


def build_all(force: bool = False):
    return build_lib(force), build_main_ksp(force), build_oracle(force)


if __name__ == "__main__":
    f = "--force" in sys.argv
    for p in build_all(f):
        print(p)
