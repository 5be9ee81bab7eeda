"""Pin the oracle's function_multiple_entries restatement to exact f(A)
entries (dense expm / coshm / sinhm) on the committed small graphs.  CPU only."""
import numpy as np
import pytest
import scipy.linalg as sla

from conftest import load_graph
from oracle import krylov_oracle as ko

EXACT = {"exp": sla.expm, "cosh": sla.coshm, "sinh": sla.sinhm}


def _omega(A, m, seed):
    S = A.tocoo()
    idx = np.random.default_rng(seed).choice(S.nnz, m, replace=False)
    om = np.stack([S.row[idx] + 1, S.col[idx] + 1], axis=1)
    return np.vstack([om, [[om[0, 0], om[0, 0]]]])   # plus one diagonal entry


@pytest.mark.parametrize("name", ["austria", "denmark", "anaheim"])
@pytest.mark.parametrize("f", ["exp", "cosh", "sinh"])
def test_fme_oracle_exact(name, f):
    A = load_graph(name)
    om = _omega(A, 10, 3)
    X, it = ko.function_multiple_entries(A, om, f, 1e-12, 80)
    E = EXACT[f](A.toarray())
    ex = np.array([E[i - 1, j - 1] for i, j in om])
    np.testing.assert_allclose(X, ex, rtol=1e-10, atol=1e-12 * np.abs(ex).max())
    assert 3 < it < 80
