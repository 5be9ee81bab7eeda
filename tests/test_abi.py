"""CPU: the C-ABI library builds, loads and exports every symbol that
include/krylov_trace.h declares; argument errors come back as statuses."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "krylov_trace.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(kt_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    fns = declared_functions()
    assert "kt_slq_trace" in fns and "kt_matrix_create_csc" in fns
    assert len(fns) >= 10


def test_library_exports_every_declared_symbol():
    from krylov_robustness_amd import _lib
    lib = _lib.load()
    bound = {name for name, _, _ in _lib.SIGNATURES}
    for name in declared_functions():
        assert hasattr(lib, name), f"{name} not exported by {_lib.LIB_PATH}"
        assert name in bound, f"{name} has no ctypes signature in _lib.SIGNATURES"


def test_abi_version_and_null_arguments():
    from krylov_robustness_amd import _lib
    lib = _lib.load()
    assert lib.kt_abi_version() == 3
    h = C.c_void_p()
    # NULL context -> KT_ERR_ARG with a message, never a crash
    st = lib.kt_matrix_create_csc(None, 0, None, None, None, 0, C.byref(h))
    assert st == _lib.KT_ERR_ARG
    assert b"NULL" in lib.kt_last_error()
    assert lib.kt_slq_trace(None, 0, 10, 0, 0, 1, 0, None, None, None) == _lib.KT_ERR_ARG
    assert lib.kt_context_destroy(None) == _lib.KT_OK


def test_matrix_create_validates_csc_before_the_device():
    """Malformed MATLAB CSC arrays are rejected on the host, before any
    device work (no GPU needed): jc[0] != 0, non-monotone jc, row indices out
    of [0, n), negative n; a valid CSC then only fails on the NULL context."""
    from krylov_robustness_amd import _lib
    lib = _lib.load()
    h = C.c_void_p()
    i64 = lambda a: (C.c_int64 * len(a))(*a)  # noqa: E731
    one = (C.c_double * 4)(1, 1, 1, 1)
    cases = [
        (2, [-1, 1, 2], [1, 0], b"start at 0"),
        (2, [0, 2, 1], [1, 0], b"monotone"),
        (2, [0, 1, 2], [1, 2], b"out of range"),
        (2, [0, 1, 2], [-1, 0], b"out of range"),
        (-1, [0], [], b"negative"),
    ]
    for n, jc, ir, msg in cases:
        st = lib.kt_matrix_create_csc(None, n, i64(jc), i64(ir or [0]), one, 0, C.byref(h))
        assert st == _lib.KT_ERR_ARG, (jc, ir)
        assert msg in lib.kt_last_error(), (jc, ir, lib.kt_last_error())
    st = lib.kt_matrix_create_csc(None, 2, i64([0, 1, 2]), i64([1, 0]), one, 0, C.byref(h))
    assert st == _lib.KT_ERR_ARG and b"NULL context" in lib.kt_last_error()


def test_no_gpu_fails_loudly():
    """With no device the library reports an error instead of computing on CPU."""
    import krylov_robustness_amd as kra
    if kra.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(kra.KrylovError):
        kra.Context(0)


def test_missing_library_raises(monkeypatch, tmp_path):
    from krylov_robustness_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.KrylovLibraryError):
        _lib.load()


def test_kt_lib_selects_the_library_and_fails_loudly(tmp_path):
    """KT_LIB names another build of the library (the A/B of compile-time
    variants); a missing one raises KrylovLibraryError naming it -- no
    fallback."""
    import subprocess
    import sys
    bad = str(tmp_path / "libkrylov_other.so")
    code = ("import krylov_robustness_amd as k, krylov_robustness_amd._lib as L\n"
            "assert k.LIB_PATH == %r\n"
            "try:\n    L.load()\nexcept L.KrylovLibraryError as e:\n    print('raised', e)\n" % bad)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT,
                       env=dict(os.environ, KT_LIB=bad))
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("raised") and bad in r.stdout


def test_every_entry_point_rejects_null_handles():
    """Every compute entry point reports KT_ERR_ARG (or another status) for a
    NULL matrix / context and NULL buffers -- never a crash -- and leaves a
    message in kt_last_error()."""
    from krylov_robustness_amd import _lib
    lib = _lib.load()
    skip = {"kt_abi_version", "kt_last_error", "kt_device_count", "kt_context_create",
            "kt_context_destroy", "kt_matrix_destroy"}
    for name, res, args in _lib.SIGNATURES:
        if name in skip:
            continue
        vals = []
        for a in args:
            if a in (C.c_int, C.c_int64, C.c_uint64):
                vals.append(1)
            elif a is C.c_double:
                vals.append(1e-8)
            elif a is _lib.REDUCE_FN:
                vals.append(_lib.REDUCE_FN(0))  # NULL callback
            else:
                vals.append(None)
        st = getattr(lib, name)(*vals)
        assert st != _lib.KT_OK, name
        assert lib.kt_last_error(), name


def _host_threads_in_child(env):
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from krylov_robustness_amd import _lib; "
            "print(_lib.load().kt_host_threads())" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return int(r.stdout.strip().splitlines()[-1])


def test_host_pool_sized_from_cpu_share_and_local_world():
    """kt_host_threads: min(16, affinity capped by the cgroup quota /
    LOCAL_WORLD_SIZE), >= 1 -- each of torchrun's ranks on a node takes its
    share of the CPUs instead of hardware_concurrency(); KT_HOST_THREADS
    overrides.  (Host-only: no GPU needed.)"""
    import os
    import sys
    sys.path.insert(0, ROOT)
    import bench
    cpus = bench.cpu_share()[0]
    base = {k: v for k, v in os.environ.items() if k not in ("KT_HOST_THREADS", "LOCAL_WORLD_SIZE")}
    for lws in (1, 2, 8):
        got = _host_threads_in_child(dict(base, LOCAL_WORLD_SIZE=str(lws)))
        assert got == max(1, min(16, cpus // lws))
    assert _host_threads_in_child(dict(base, KT_HOST_THREADS="3", LOCAL_WORLD_SIZE="8")) == 3
