"""CPU check of the algebra behind the y-form hot path (kt_kernels.hip
k_spmm_lanczos / k_ycoef): the A-image recurrence
y_{j+1} = (A y_j - alpha_j y_j - beta_j y_{j-1}) / beta_{j+1} with alpha, beta
from the Gram identities reproduces the oracle's CGS2-window Lanczos
(oracle/slq_ref.c, lanczos_krylov.m:73-115) quadratures, and the guard ratio
beta_k^2 / ||y_{k-1}||^2 separates healthy runs from a lucky breakdown.
NumPy restatement of the device recurrence (test code only)."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import load_graph
from oracle import krylov_oracle as ko
from oracle import slq_ref

GUARD = 1e-4  # kt_slq.cpp kYformGuard


def yform(A, z, m):
    """Returns (alpha, beta, min guard ratio) as k_spmm_lanczos + k_ycoef form them."""
    v0 = z / np.linalg.norm(z)
    y = A @ v0
    ym1 = np.zeros_like(y)
    alpha, beta = [v0 @ y], []
    ny2, yd, aprev, b = y @ y, 0.0, 0.0, 0.0
    ratio = np.inf
    for j in range(m - 1):
        a = alpha[j]
        b1sq = ny2 - a * a - b * b
        ratio = min(ratio, b1sq / ny2)
        b1 = np.sqrt(max(b1sq, 0.0))
        t = A @ y
        ynew = (t - a * y - b * ym1) / b1
        anew = (y @ t - 2 * a * ny2 - 2 * b * yd + a ** 3 + 2 * a * b * b + b * b * aprev) / b1sq
        yd, ny2, aprev, b = y @ ynew, ynew @ ynew, a, b1
        ym1, y = y, ynew
        alpha.append(anew)
        beta.append(b1)
    return np.array(alpha), np.array(beta), ratio


def quad(alpha, beta, fun):
    T = np.diag(alpha) + np.diag(beta, 1) + np.diag(beta, -1)
    th, Z = np.linalg.eigh(T)
    return float(np.sum(Z[0] ** 2 * getattr(np, fun)(th)))


@pytest.mark.parametrize("name", ["oregon_A0", "denmark", "india", "rome"])
@pytest.mark.parametrize("m,fun", [(20, "exp"), (30, "sinh"), (60, "exp")])
def test_yform_matches_cgs2_oracle(name, m, fun):
    A = load_graph(name)
    n = A.shape[0]
    if m >= n:
        pytest.skip("m >= n")
    _, q_ref = slq_ref.slq_trace(A, 4, m, seed=7, fun=fun)
    Z = ko.rademacher(n, np.arange(4), 7)
    for p in range(4):
        al, be, ratio = yform(A, Z[:, p], m)
        assert ratio > GUARD  # healthy run: the guard does not trip
        q = n * quad(al, be, fun)
        assert q == pytest.approx(q_ref[p], rel=1e-10)


@pytest.mark.filterwarnings("ignore::RuntimeWarning")
def test_yform_guard_trips_on_breakdown():
    """K_20: the Krylov space of a generic z has dimension 2, so beta_2 ~ 0
    and the guard ratio falls to rounding level -- the device sends such a
    sweep to the explicit CGS2 sweep."""
    A = sp.csr_matrix(np.ones((20, 20)) - np.eye(20))
    z = ko.rademacher(20, np.arange(1), 3)[:, 0]
    _, _, ratio = yform(A, z, 4)
    assert not ratio > GUARD
