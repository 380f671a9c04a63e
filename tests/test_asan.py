"""The library's host-side C/C++ (operand producers, MPIAIJ split, host GAMG
set-up, the oracle's C MatMult) under AddressSanitizer and UBSan (SURVEY.md
§5). CPU only: GPU code is not sanitised on this pool."""
import shutil
import subprocess

import pytest

from conftest import ROOT


def test_host_code_is_asan_ubsan_clean(tmp_path):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("no g++")
    csrc = ROOT / "petsc-openacc_amd" / "csrc"
    exe = tmp_path / "host_checks"
    flags = ["-O1", "-g", "-std=c++17", "-fopenmp", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
             "-fno-sanitize-recover=undefined", f"-I{ROOT / 'include'}", f"-I{csrc}"]
    objs = []
    c_obj = tmp_path / "oracle.o"
    subprocess.run(["gcc", "-O1", "-g", "-fopenmp", "-fsanitize=address,undefined", "-ffp-contract=off", "-c",
                    str(ROOT / "oracle" / "matmult_seqaij.c"), "-o", str(c_obj)], check=True)
    objs.append(str(c_obj))
    r = subprocess.run([gxx, *flags, str(ROOT / "tests" / "asan" / "host_checks.cpp"), str(csrc / "harness.cpp"),
                        str(csrc / "gamg_setup.cpp"), *objs, "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                         env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "OMP_NUM_THREADS": "4",
                              "PATH": "/usr/bin:/bin"})
    assert run.returncode == 0, run.stderr[-4000:]
    assert "host checks ok" in run.stdout
    assert "AddressSanitizer" not in run.stderr and "runtime error" not in run.stderr
