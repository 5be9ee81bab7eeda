"""CPU: the MEX drop-in shim (krylov_robustness_amd/mex/kt_mex.cpp) compiles for
every entry point against a stub of MATLAB's mex.h (type check only: MATLAB
is absent, so the shim is source-only; its C-ABI calls are exercised by the
ctypes tests)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

ENTRIES = ["TRACE_EXP", "MC_TRACE", "TRACE_FUN_UPDATE", "FUN_UPDATE", "FG_EXP", "FG_FUN",
           "KRYLOV_MIOBI", "FME", "HESS_EXP", "HESS_FUN"]


@pytest.mark.parametrize("entry", ENTRIES)
def test_mex_shim_compiles(entry, tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    src = os.path.join(ROOT, "krylov_robustness_amd", "mex", "kt_mex.cpp")
    r = subprocess.run([gxx, "-std=c++17", "-fsyntax-only", "-Wall", f"-DKT_ENTRY_{entry}",
                        "-I", os.path.join(ROOT, "tests", "mexstub"), src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("entry", ENTRIES)
def test_mex_entry_library_exports_mexfunction(entry):
    """The per-entry builds against the stand-in runtime (make -C tests/mexstub,
    run by __graft_entry__.build()) load next to libkrylov_hip.so and export
    mexFunction with C linkage, as MATLAB's loader looks it up.  No call is
    made here (no GPU); tests/test_mex_exec.py runs them on the GPU box."""
    import ctypes
    from krylov_robustness_amd import _lib
    # KT_MEXSTUB_BUILD: the sanitizer build's directory (tools/sanitize.sh)
    build = os.environ.get("KT_MEXSTUB_BUILD") or os.path.join(ROOT, "tests", "mexstub", "_build")
    if not os.path.exists(os.path.join(build, f"kt_mex_{entry}.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "mexstub")], check=True,
                       capture_output=True)
    _lib.load()
    ctypes.CDLL(os.path.join(build, "libmexstub.so"), mode=ctypes.RTLD_GLOBAL)
    lib = ctypes.CDLL(os.path.join(build, f"kt_mex_{entry}.so"))
    assert hasattr(lib, "mexFunction")
