"""The C + OpenMP restatement of the reference's own trace_exp composition
(oracle/mctrace_ref.c: mc_trace.m + expmv.m + select_taylor_degree.m +
normAm.m), used as the CPU baseline of bench.py's reference-composition leg,
against the numpy restatement (oracle/krylov_oracle.py) it must equal: the
same s, m, mv and F (the same operations in the same order per row), and
the same trace_exp estimate and round count."""
import numpy as np
import pytest

from conftest import load_graph
from oracle import krylov_oracle as ko
from oracle import mctrace_ref as mr


@pytest.mark.parametrize("name", ["oregon_A0", "rome", "india"])
def test_expmv_equals_numpy_restatement(name):
    A = load_graph(name).tocsr()
    B = ko.rademacher(A.shape[0], range(10), 3)
    F, s, m, mv, st = mr.expmv(1.0, A, B, nthreads=4)
    Fo, so, mo, mvo = ko.expmv(1.0, A, B)
    assert (s, m, mv) == (so, mo, mvo)
    np.testing.assert_allclose(F, Fo, rtol=1e-14, atol=1e-14 * np.abs(Fo).max())
    assert st["calls"] == 1 and 0 < st["terms"] <= s * m


@pytest.mark.parametrize("name", ["oregon_A0", "india"])
def test_trace_exp_equals_numpy_restatement(name):
    A = load_graph(name).tocsr()
    tr, res, it, st = mr.trace_exp(A, seed=1, nthreads=4)
    tro, reso, ito = ko.mc_trace(lambda x: ko.expmv(1.0, A, x)[0], A.shape[0], 1e-4, 1000, 1, seed=1)
    assert it == ito
    assert tr == pytest.approx(tro, rel=1e-12)
    assert res == pytest.approx(reso, rel=1e-6, abs=1e-12)
    assert st["calls"] == 3 * it  # three Afun calls per round (mc_trace.m:45, :46, :49)


def test_rejects_what_it_does_not_restate():
    import scipy.sparse as sp
    A = load_graph("oregon_A0").tolil()
    A[0, 0] = 1.0  # a self loop: mu > 0, A - mu I has negative entries (normest1 branch)
    with pytest.raises(ValueError):
        mr.expmv(1.0, sp.csr_matrix(A), np.ones((A.shape[0], 10)))


def test_round_host_times_positive():
    t_qr, t_proj = mr.round_host_times(20000, nthreads=2)
    assert t_qr > 0 and t_proj > 0
