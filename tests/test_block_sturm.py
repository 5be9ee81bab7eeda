"""CPU check of the block Sturm count that k_pair_fused uses for the greedy
candidates' projected eigenproblems (kt_pairs.hip block_count_ms): a numpy
restatement of the same recurrence -- D_0 = M_0 - xI, D_{k+1} = M_{k+1} - xI
- U_k' D_k^{-1} U_k, count = negatives of every 2x2 D_k, a near-singular D_k
evaluated at x + eps -- bisected to 2 ulp of the spectral radius and compared
with LAPACK eigvalsh on the symmetrised block-tridiagonal projections
(tGm, Gm) that the oracle's trace_fun_update (trace_fun_update.m:71-84)
forms for India greedy candidates, and on a projection whose leading block
is zero with the shift exactly 0 (the case a determinant-only perturbation
gets wrong)."""
import numpy as np
import pytest

from conftest import load_graph
from oracle import krylov_oracle as ko

PIVMIN0 = 2.2250738585072014e-308


def blocks(M):
    j = M.shape[0] // 2
    Mb = [(M[2 * k, 2 * k], M[2 * k + 1, 2 * k], M[2 * k + 1, 2 * k + 1]) for k in range(j)]
    Ub = [(M[2 * k, 2 * k + 2], M[2 * k, 2 * k + 3], M[2 * k + 1, 2 * k + 2], M[2 * k + 1, 2 * k + 3])
          for k in range(j - 1)]
    return Mb, Ub


def count(Mb, Ub, x, pivmin):
    eps = 10.0 * np.sqrt(pivmin)
    cnt = 0
    a, b, c = Mb[0][0] - x, Mb[0][1], Mb[0][2] - x
    for k in range(len(Mb)):
        det = a * c - b * b
        if abs(det) < pivmin:
            a, c = a - eps, c - eps
            det = a * c - b * b
            if abs(det) < pivmin:
                det = -pivmin
        cnt += 1 if det < 0 else (2 if a < 0 else 0)
        if k + 1 == len(Mb):
            break
        u0, u1, u2, u3 = Ub[k]
        i00, i01, i11 = c / det, -b / det, a / det
        t00, t01 = i00 * u0 + i01 * u2, i00 * u1 + i01 * u3
        t10, t11 = i01 * u0 + i11 * u2, i01 * u1 + i11 * u3
        s00, s01, s11 = u0 * t00 + u2 * t10, u0 * t01 + u2 * t11, u1 * t01 + u3 * t11
        a, b, c = Mb[k + 1][0] - x - s00, Mb[k + 1][1] - s01, Mb[k + 1][2] - x - s11
    return cnt


def eigs_block_sturm(M):
    Mb, Ub = blocks(M)
    off = np.abs(M).sum(1) - np.abs(np.diag(M))
    lo, hi = (np.diag(M) - off).min(), (np.diag(M) + off).max()
    pivmin = PIVMIN0 * max(1.0, np.abs(M).max()) ** 4
    out = []
    for k in range(M.shape[0]):
        a, b = lo, hi
        while b - a > 4.4e-16 * max(abs(lo), abs(hi)):
            m = 0.5 * (a + b)
            if m in (a, b):
                break
            if count(Mb, Ub, m, pivmin) > k:
                b = m
            else:
                a = m
        out.append(0.5 * (a + b))
    return np.array(out)


def projections(A, U, B, tol, it):
    """(tGm, Gm) of the oracle's last step, symmetrised as the reference does."""
    cap = []
    orig = np.linalg.eigvalsh

    def spy(M, *a, **k):
        cap.append(np.array(M))
        return orig(M, *a, **k)
    np.linalg.eigvalsh = spy
    try:
        ko.trace_fun_update(A, U, B, tol, it)
    finally:
        np.linalg.eigvalsh = orig
    return cap[-2], cap[-1]


def test_block_sturm_matches_eigvalsh_on_greedy_projections():
    import krylov_robustness_amd as kra
    A = load_graph("india")
    n = A.shape[0]
    E = kra.find_top_edges(A, kra.compute_centrality(A), 40, "min")
    B = -np.array([[0.0, 1.0], [1.0, 0.0]])
    for h in range(0, 40, 4):
        U = np.zeros((n, 2))
        U[E[h][0] - 1, 0] = 1
        U[E[h][1] - 1, 1] = 1
        for M in projections(A, U, B, 1e-10, 100):
            ref = np.linalg.eigvalsh(M)
            got = eigs_block_sturm(M)
            assert np.abs(got - ref).max() <= 2e-14 * max(1.0, np.abs(ref).max()), h


def test_block_sturm_zero_leading_block_at_zero_shift():
    """M_0 = 0 with a Gershgorin interval symmetric about 0: the first
    bisection point is x = 0, where D_0 = 0 has a zero adjugate."""
    rng = np.random.default_rng(0)
    j = 6
    M = np.zeros((2 * j, 2 * j))
    for k in range(j):
        if k:
            d = rng.normal(size=(2, 2))
            M[2 * k:2 * k + 2, 2 * k:2 * k + 2] = d + d.T
        if k + 1 < j:
            u = rng.normal(size=(2, 2))
            M[2 * k:2 * k + 2, 2 * k + 2:2 * k + 4] = u
            M[2 * k + 2:2 * k + 4, 2 * k:2 * k + 2] = u.T
    Mb, Ub = blocks(M)
    pivmin = PIVMIN0 * max(1.0, np.abs(M).max()) ** 4
    ref = np.linalg.eigvalsh(M)
    assert count(Mb, Ub, 0.0, pivmin) == int((ref < 0).sum() + (ref == 0).sum())
    np.testing.assert_allclose(eigs_block_sturm(M), ref, atol=2e-14 * np.abs(ref).max())


def count_newton(Mb, Ub, x, pivmin):
    """block_count_newton (kt_pairs.hip): the count and S = d/dx log|det(M - xI)|
    = sum_k tr(D_k^{-1} D_k'), D_0' = -I, D_{k+1}' = -I + T_k' D_k' T_k,
    T_k = D_k^{-1} U_k."""
    eps = 10.0 * np.sqrt(pivmin)
    cnt, S = 0, 0.0
    a, b, c = Mb[0][0] - x, Mb[0][1], Mb[0][2] - x
    p, q, r = -1.0, 0.0, -1.0
    for k in range(len(Mb)):
        det = a * c - b * b
        if abs(det) < pivmin:
            a, c = a - eps, c - eps
            det = a * c - b * b
            if abs(det) < pivmin:
                det = -pivmin
        cnt += 1 if det < 0 else (2 if a < 0 else 0)
        i00, i01, i11 = c / det, -b / det, a / det
        S += i00 * p + 2 * i01 * q + i11 * r
        if k + 1 == len(Mb):
            break
        u0, u1, u2, u3 = Ub[k]
        t00, t01 = i00 * u0 + i01 * u2, i00 * u1 + i01 * u3
        t10, t11 = i01 * u0 + i11 * u2, i01 * u1 + i11 * u3
        s00, s01, s11 = u0 * t00 + u2 * t10, u0 * t01 + u2 * t11, u1 * t01 + u3 * t11
        e00, e01 = p * t00 + q * t10, p * t01 + q * t11
        e10, e11 = q * t00 + r * t10, q * t01 + r * t11
        p, q, r = -1.0 + t00 * e00 + t10 * e10, t00 * e01 + t10 * e11, -1.0 + t01 * e01 + t11 * e11
        a, b, c = Mb[k + 1][0] - x - s00, Mb[k + 1][1] - s01, Mb[k + 1][2] - x - s11
    return cnt, S


def eigs_block_newton(M, stats):
    """wave_multisect_blk's default path: bracket to span/4096 by counts, then
    safeguarded Newton on det(M - xI) (accepted at a step <= 64 atol),
    certified by the counts at x -+ 8 atol; uncertified eigenvalues are
    bisected on to atol from the bracket Newton left."""
    Mb, Ub = blocks(M)
    nn = M.shape[0]
    off = np.abs(M).sum(1) - np.abs(np.diag(M))
    lo, hi = (np.diag(M) - off).min(), (np.diag(M) + off).max()
    span = hi - lo
    lo, hi = lo - 2.2e-16 * span, hi + 2.2e-16 * span
    pivmin = PIVMIN0 * max(1.0, np.abs(M).max()) ** 4
    atol = 4.4e-16 * max(abs(lo), abs(hi))
    out = []
    for k in range(nn):
        a, b = lo, hi
        while b - a > (hi - lo) / 4096:
            m = 0.5 * (a + b)
            if count(Mb, Ub, m, pivmin) > k:
                b = m
            else:
                a = m
        x, conv = 0.5 * (a + b), False
        for _ in range(8):
            cnt, S = count_newton(Mb, Ub, x, pivmin)
            if cnt > k:
                b = x
            else:
                a = x
            with np.errstate(all="ignore"):
                xn = x - 1.0 / S
            inb = a <= xn <= b
            if abs(xn - x) <= 64 * atol or not b - a > atol:
                conv = True
                x = xn if inb else x
                break
            x = xn if inb else 0.5 * (a + b)
        if conv and count(Mb, Ub, x - 8 * atol, pivmin) <= k < count(Mb, Ub, x + 8 * atol, pivmin):
            stats["certified"] += 1
            out.append(x)
            continue
        while b - a > atol:
            m = 0.5 * (a + b)
            if m in (a, b):
                break
            if count(Mb, Ub, m, pivmin) > k:
                b = m
            else:
                a = m
        out.append(0.5 * (a + b))
    stats["total"] += nn
    return np.array(out)


def test_block_newton_matches_eigvalsh_on_greedy_projections():
    """The Newton-accelerated multisection of k_pair_fused / k_pair_eig_blk
    (KT_BLK_NEWTON): same eigenvalues as eigvalsh to 2e-14 of the spectral
    radius, and nearly every eigenvalue certified without the fallback."""
    import krylov_robustness_amd as kra
    A = load_graph("india")
    n = A.shape[0]
    E = kra.find_top_edges(A, kra.compute_centrality(A), 40, "min")
    B = -np.array([[0.0, 1.0], [1.0, 0.0]])
    st = {"certified": 0, "total": 0}
    for h in range(0, 40, 4):
        U = np.zeros((n, 2))
        U[E[h][0] - 1, 0] = 1
        U[E[h][1] - 1, 1] = 1
        for M in projections(A, U, B, 1e-10, 100):
            ref = np.linalg.eigvalsh(M)
            got = eigs_block_newton(M, st)
            assert np.abs(got - ref).max() <= 2e-14 * max(1.0, np.abs(ref).max()), h
    assert st["certified"] >= 0.95 * st["total"], st


def test_count_newton_derivative_matches_finite_difference():
    rng = np.random.default_rng(1)
    j = 5
    M = np.zeros((2 * j, 2 * j))
    for k in range(j):
        d = rng.normal(size=(2, 2))
        M[2 * k:2 * k + 2, 2 * k:2 * k + 2] = d + d.T
        if k + 1 < j:
            u = rng.normal(size=(2, 2))
            M[2 * k:2 * k + 2, 2 * k + 2:2 * k + 4] = u
            M[2 * k + 2:2 * k + 4, 2 * k:2 * k + 2] = u.T
    Mb, Ub = blocks(M)
    lam = np.linalg.eigvalsh(M)
    for x in (-7.3, 0.1234, 2.5):
        cnt, S = count_newton(Mb, Ub, x, PIVMIN0)
        assert cnt == int((lam < x).sum())
        assert S == pytest.approx(float(np.sum(1.0 / (x - lam))), rel=1e-10)
