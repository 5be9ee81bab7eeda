"""CPU: the MEX shim's argument decoding (krylov_robustness_amd/mex/kt_mex.cpp)
EXECUTED without a GPU, through the stand-in MEX runtime (tests/mexstub):
MATLAB CSC (mwIndex jc / ir) and full matrices decoded and compressed,
non-square and non-double A refused with the reference's messages, too few
arguments refused per entry.  With no device the first library call that
needs one (the context) fails, and the shim must turn that into a MATLAB
error, not a crash; on a GPU host the same calls succeed.  tools/sanitize.sh
runs this module (with the rest of the CPU suite) against ASan + UBSan
builds of the shim, the stub runtime and the library."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_graph
from test_mex_exec import ENTRIES, Mex, MexRaised


@pytest.fixture(scope="module")
def mex():
    return Mex()


def _device_or_context_error(mex, *args):
    try:
        out = mex.call("TRACE_EXP", 1, *args)
    except MexRaised as e:  # no GPU here: the context (or the matrix upload) fails cleanly
        assert e.ident in ("krylov_hip:context", "krylov_hip:matrix"), (e.ident, e.msg)
        return None
    assert np.isfinite(out[0])
    return out[0]


def test_sparse_and_full_a_decode(mex):
    A = load_graph("oregon_A0")
    _device_or_context_error(mex, A)                   # CSC, mwIndex jc / ir
    _device_or_context_error(mex, A[:60, :60].toarray())  # full: compressed column by column
    _device_or_context_error(mex, sp.csc_matrix((5, 5)))  # no entries


def test_non_square_and_non_double_a_refused(mex):
    with pytest.raises(MexRaised) as e:
        mex.call("TRACE_EXP", 1, sp.random(6, 5, density=0.5, random_state=1, format="csc"))
    assert e.value.ident == "krylov_hip:A" and e.value.msg == "The matrix A should be square"
    with pytest.raises(MexRaised) as e:
        mex.call("TRACE_EXP", 1, "not a matrix")
    assert e.value.ident == "krylov_hip:A" and "real double" in e.value.msg
    # fun_and_grad_krylov_*: ishermitian(A) is the reference's first test
    X = np.zeros(3)
    Om = np.array([[1.0, 2.0], [2.0, 3.0], [1.0, 3.0]])
    for entry, extra in (("FG_EXP", (Om, 1.0, 1e-8, 10)),):
        with pytest.raises(MexRaised) as e:
            mex.call(entry, 2, X, sp.random(6, 5, density=0.5, random_state=2, format="csc"), *extra)
        assert "not Hermitian" in e.value.msg


@pytest.mark.parametrize("entry", ENTRIES)
def test_too_few_arguments_refused(mex, entry):
    with pytest.raises(MexRaised) as e:
        mex.call(entry, 1)
    assert e.value.ident == "krylov_hip:nargin"
