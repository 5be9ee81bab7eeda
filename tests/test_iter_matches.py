"""The iteration-count rule the GPU parity tests use (conftest.iter_matches):
exact agreement, or one step apart only where the oracle's lag-2 stop test
(trace_fun_update.m:104-118) was marginal at the disagreeing step."""
from conftest import iter_matches
from oracle import krylov_oracle as ko
from conftest import load_graph
import numpy as np


def test_exact_and_marginal_rule():
    tol = 1e-12
    hist = [(3, 5e-10, 10.0), (4, 1.00000000001e-12, 10.0), (5, 1e-15, 10.0)]
    assert iter_matches(5, 5, hist, tol)
    assert iter_matches(4, 5, hist, tol)        # step 4 marginal: |err - tol| ~ 1e-23 << 1e-11 * 10
    assert not iter_matches(3, 4, hist, tol)    # step 3 was far from tol
    assert not iter_matches(3, 5, hist, tol)    # two steps apart never
    assert not iter_matches(4, 5, [], tol)


def test_oracle_history_matches_its_iteration_count():
    A = load_graph("rome")
    n = A.shape[0]
    U = np.zeros((n, 2)); U[0, 0] = 1; U[5, 1] = 1
    B = -np.array([[0.0, 1.0], [1.0, 0.0]])
    hist = []
    _, it, lucky = ko.trace_fun_update(A, U, B, 1e-12, 100, 0, "exp", hist=hist)
    assert hist[0][0] == 3 and [h[0] for h in hist] == list(range(3, it + 1))
    if not lucky and it < 100:
        assert hist[-1][1] < 1e-12 and all(h[1] >= 1e-12 for h in hist[:-1])
