"""GPU parity for mc_trace / trace_exp / expmv / the Lanczos-f Afun (SURVEY.md
§8a rows a1, a2, a3, a10) against the oracle on the same counter-RNG probes.
Tolerances: 1e-9 relative where the device runs the reference algorithm
(expmv Taylor loop, matrix Afun); 1e-6 for the Lanczos Afun inside mc_trace,
where the device evaluates trace(Q' f(A) Q) as Gauss quadratures while the
oracle forms the literal vectors f(A)Q ~= ||q|| V f(T) e1 (equal up to the
loss of Lanczos orthogonality)."""
import numpy as np
import pytest

from conftest import load_graph
from oracle import krylov_oracle as ko

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kra():
    import krylov_robustness_amd as kra
    return kra


@pytest.mark.parametrize("name", ["anaheim", "oregon_A0", "austria"])
def test_expmv_matches_oracle(kra, gpu_ctx, name):
    A = load_graph(name)
    b = np.random.default_rng(1).normal(size=(A.shape[0], 3))
    F, s, m, mv = kra.expmv(1.0, kra.DeviceMatrix(A, gpu_ctx), b, ctx=gpu_ctx)
    Fo, so, mo, mvo = ko.expmv(1.0, A, b)
    assert (s, m, mv) == (so, mo, mvo)  # mv: the device-side stop fires at the oracle's term
    np.testing.assert_allclose(F, Fo, rtol=1e-11, atol=1e-13 * np.abs(Fo).max())


def test_expmv_wide_block_and_unfused_form(kra, gpu_ctx, monkeypatch):
    """Blocks wider than 32 columns run the four-launch Taylor term (block SpMM
    + combine + k_expmv_term + k_expmv_check); KT_EXPMV_UNFUSED=1 selects it
    for narrow blocks too.  Both agree with the oracle and with the fused
    k_expmv_step (same s, m, mv; 1e-13)."""
    A = load_graph("oregon_A0")
    D = kra.DeviceMatrix(A, gpu_ctx)
    b = np.random.default_rng(3).normal(size=(A.shape[0], 40))
    F, s, m, mv = kra.expmv(1.0, D, b, ctx=gpu_ctx)
    Fo, so, mo, mvo = ko.expmv(1.0, A, b)
    assert (s, m, mv) == (so, mo, mvo)
    np.testing.assert_allclose(F, Fo, rtol=1e-11, atol=1e-13 * np.abs(Fo).max())
    b3 = b[:, :3]
    Ff, *rf = kra.expmv(1.0, D, b3, ctx=gpu_ctx)
    monkeypatch.setenv("KT_EXPMV_UNFUSED", "1")
    Fu, *ru = kra.expmv(1.0, D, b3, ctx=gpu_ctx)
    assert rf == ru
    np.testing.assert_allclose(Fu, Ff, rtol=1e-13, atol=1e-15 * np.abs(Ff).max())


def _expmv_graph(graph):
    from krylov_robustness_amd import graphs
    if graph == "er100k":
        return graphs.erdos_renyi(100_000, 500_000, seed=0)
    if graph.startswith("chunglu200k"):
        # scale-free: 17-64-degree rows (one wave each in the split forms) and
        # rows of degree > 64 (a workgroup each in the split kernel, four
        # chain sets of one wave in the row-blocked one); "_w": fp64 weights
        A = graphs.chung_lu(200_000, 2_000_000, gamma=2.5, seed=3)
        if graph.endswith("_w"):
            import scipy.sparse as sp
            U = sp.triu(A, 1).tocoo()
            w = np.random.default_rng(4).uniform(0.5, 1.5, size=U.nnz)
            W = sp.coo_matrix((w, (U.row, U.col)), shape=A.shape)
            A = (W + W.T).tocsr()
            A.sort_indices()
        return A
    return load_graph(graph)


@pytest.mark.parametrize("graph", ["oregon_A6", "er100k", "chunglu200k", "chunglu200k_w"])
def test_expmv_split_check_form(kra, gpu_ctx, monkeypatch, graph):
    """Grids above 1,024 workgroups run the SPLIT term (the stop test in its
    own one-wave launch after each term, a stopped term returning before its
    gathers) instead of the fused one; the split term runs row-blocked
    (k_expmv_rows, resident workgroups, round 6) unless KT_EXPMV_ROWS=0
    selects the workgroup-per-row-class split kernel; KT_EXPMV_SORTWIN sets
    the short-row order (a row-build option: the matrix is rebuilt per
    form below).  On oregon_A6 (340 workgroups, fused by default), ER
    n = 100k (3,125, split) and Chung-Lu n = 200k (medium and long rows; unit
    and fp64 weights) all four forms give the same F, s, m, mv bit for bit,
    and agree with the oracle; the first column alone (P = 1) too."""
    A = _expmv_graph(graph)
    b = np.random.default_rng(7).normal(size=(A.shape[0], 10))
    # (KT_EXPMV_SPLIT, KT_EXPMV_ROWS, KT_EXPMV_SORTWIN, KT_EXPMV_ROWCHECK):
    # fused; split; row-blocked (short rows degree-sorted in windows of 4,096
    # rows, each term testing the previous term's stop: the default);
    # row-blocked with the whole matrix's short rows degree-sorted; row-blocked
    # with the separate slot-check launch
    forms = (("0", None, None, None), ("1", "0", None, None), ("1", None, None, None), ("1", None, "0", None),
             ("1", None, None, "0"))
    keys = ("KT_EXPMV_SPLIT", "KT_EXPMV_ROWS", "KT_EXPMV_SORTWIN", "KT_EXPMV_ROWCHECK")
    for B in (b, b[:, :1]):
        outs = []
        for f in forms:
            for k, v in zip(keys, f):
                if v is None:
                    monkeypatch.delenv(k, raising=False)
                else:
                    monkeypatch.setenv(k, v)
            Df = kra.DeviceMatrix(A, gpu_ctx)  # the natural CSR (and its task lists) built under f
            outs.append(kra.expmv(1.0, Df, B, ctx=gpu_ctx))
            Df.close()
        for k in keys:
            monkeypatch.delenv(k, raising=False)
        for o in outs[1:]:
            assert tuple(outs[0][1:]) == tuple(o[1:])
            assert np.array_equal(outs[0][0], o[0])
        Fo, *ro = ko.expmv(1.0, A, B)
        assert tuple(outs[0][1:]) == tuple(ro)
        np.testing.assert_allclose(outs[0][0], Fo, rtol=1e-11, atol=1e-13 * np.abs(Fo).max())


@pytest.mark.parametrize("name,loops", [("oregon_A6", False), ("oregon_A0", True), ("anaheim", False)])
def test_expmv_per_term_launches_match_oracle(kra, gpu_ctx, name, loops):
    """The per-term launches (k_expmv_step) give the oracle's F with equal s,
    m and mv; self loops exercise mu != 0."""
    from test_normest1 import looped
    A = load_graph(name)
    if loops:
        A = looped(A)
    D = kra.DeviceMatrix(A, gpu_ctx)
    b = np.random.default_rng(5).normal(size=(A.shape[0], 10))
    ref = kra.expmv(1.0, D, b, ctx=gpu_ctx)
    Fo, *ro = ko.expmv(1.0, A, b)
    assert tuple(ref[1:]) == tuple(ro)
    np.testing.assert_allclose(ref[0], Fo, rtol=1e-11, atol=1e-13 * np.abs(Fo).max())


def test_expmv_host_stop_flag_is_exact(kra, gpu_ctx, monkeypatch):
    """The per-term launches stop being queued once the launch that found a
    stage's stop test satisfied has told the host (coherent host flag): the
    skipped launches were no-ops, so F, s, m, mv equal queueing all s * m
    terms (KT_EXPMV_STOPFLAG=0), bit for bit; trace_exp likewise."""
    A = load_graph("oregon_A6")
    D = kra.DeviceMatrix(A, gpu_ctx)
    b = np.random.default_rng(9).normal(size=(A.shape[0], 10))
    f1 = kra.expmv(1.0, D, b, ctx=gpu_ctx)
    t1 = kra.trace_exp(D, method="expmv", seed=2, ctx=gpu_ctx)
    monkeypatch.setenv("KT_EXPMV_STOPFLAG", "0")
    f0 = kra.expmv(1.0, D, b, ctx=gpu_ctx)
    t0 = kra.trace_exp(D, method="expmv", seed=2, ctx=gpu_ctx)
    assert tuple(f1[1:]) == tuple(f0[1:])
    np.testing.assert_array_equal(f1[0], f0[0])
    assert t1 == t0


def test_lanczos_fmv_matches_oracle(kra, gpu_ctx):
    A = load_graph("rome")
    X = np.random.default_rng(2).normal(size=(A.shape[0], 4))
    Y = kra.lanczos_fmv(kra.DeviceMatrix(A, gpu_ctx), X, m=20, fun="exp", ctx=gpu_ctx)
    Yo = ko.lanczos_fmv(A, X, 20, "exp")
    np.testing.assert_allclose(Y, Yo, rtol=1e-8, atol=1e-10 * np.abs(Yo).max())


def test_lanczos_fmv_yform_basis_matches_oracle(kra, gpu_ctx, monkeypatch):
    """f(A) x with the Lanczos basis formed by the y-form pass itself (KF_VB:
    v_{j+1} = g y_j - a v_j - b v_{j-1} with the pass's own coefficients;
    KT_LC_YBASIS=1 routes lanczos_fmv through it): 4 columns and 40 columns
    (three 16-wide sweeps, the last padded) match the oracle and the explicit
    CGS2 sweep's result.  A column that is an eigenvector of A (a lucky
    breakdown at step 1) trips the y-form guard: its sweep is redone whole by
    the explicit sweep with its basis, still matching the oracle."""
    import scipy.sparse.linalg as sla
    A = load_graph("rome")
    D = kra.DeviceMatrix(A, gpu_ctx)
    for ncol, seed in ((4, 2), (40, 5)):
        X = np.random.default_rng(seed).normal(size=(A.shape[0], ncol))
        Ye = kra.lanczos_fmv(D, X, m=20, fun="exp", ctx=gpu_ctx)
        monkeypatch.setenv("KT_LC_YBASIS", "1")
        Y = kra.lanczos_fmv(D, X, m=20, fun="exp", ctx=gpu_ctx)
        monkeypatch.delenv("KT_LC_YBASIS")
        Yo = ko.lanczos_fmv(A, X, 20, "exp")
        np.testing.assert_allclose(Y, Yo, rtol=1e-8, atol=1e-10 * np.abs(Yo).max())
        np.testing.assert_allclose(Y, Ye, rtol=1e-9, atol=1e-11 * np.abs(Ye).max())
    w, v = sla.eigsh(A.astype(np.float64), k=1, which="LA")
    X = np.random.default_rng(9).normal(size=(A.shape[0], 3))
    X[:, 1] = v[:, 0]
    before = gpu_ctx.stat(0)
    monkeypatch.setenv("KT_LC_YBASIS", "1")
    Y = kra.lanczos_fmv(D, X, m=20, fun="exp", ctx=gpu_ctx)
    monkeypatch.delenv("KT_LC_YBASIS")
    assert gpu_ctx.stat(0) > before  # the explicit redo ran
    Yo = ko.lanczos_fmv(A, X, 20, "exp")
    np.testing.assert_allclose(Y, Yo, rtol=1e-8, atol=1e-10 * np.abs(Yo).max())


def test_mc_trace_s_term_yform_basis(kra, gpu_ctx, monkeypatch):
    """mc_trace with the Lanczos Afun can form the lone S term's f(A) S with
    the basis-forming y-form sweep (KT_MC_YBASIS=1) instead of the explicit
    sweep (the default): the same rounds and the estimate to 1e-11."""
    A = load_graph("oregon_A0")
    D = kra.DeviceMatrix(A, gpu_ctx)
    kw = dict(tol=1e-6, maxit=120, isAreal=1, seed=3, fun="exp", m=20)
    ref = kra.mc_trace("lanczos", None, A=D, ctx=gpu_ctx, **kw)
    monkeypatch.setenv("KT_MC_YBASIS", "1")
    got = kra.mc_trace("lanczos", None, A=D, ctx=gpu_ctx, **kw)
    monkeypatch.delenv("KT_MC_YBASIS")
    assert got[2] == ref[2]
    assert got[0] == pytest.approx(ref[0], rel=1e-11)


def test_lanczos_fmv_many_columns_over_lanes(kra, gpu_ctx):
    """40 columns: three 16-wide explicit sweeps (the last zero-padded) queued
    step by step on three sweep lanes (kt_slq.cpp lanczos_columns_split).
    Every column matches the oracle, and a column's f(A) x is bit-identical
    to the same column computed in a call of its own sweep alone (its form
    depends only on its sweep's width, not on the lanes beside it)."""
    A = load_graph("rome")
    X = np.random.default_rng(5).normal(size=(A.shape[0], 40))
    D = kra.DeviceMatrix(A, gpu_ctx)
    Y = kra.lanczos_fmv(D, X, m=20, fun="exp", ctx=gpu_ctx)
    Yo = ko.lanczos_fmv(A, X, 20, "exp")
    np.testing.assert_allclose(Y, Yo, rtol=1e-8, atol=1e-10 * np.abs(Yo).max())
    Y16 = kra.lanczos_fmv(D, np.ascontiguousarray(X[:, 16:32]), m=20, fun="exp", ctx=gpu_ctx)
    np.testing.assert_array_equal(Y[:, 16:32], Y16)


@pytest.mark.parametrize("name", ["denmark", "anaheim"])
def test_mc_trace_matrix_afun(kra, gpu_ctx, name):
    """mc_trace.m:32-34 (Afun is a matrix), 3 rounds of nested deflation."""
    A = load_graph(name)
    tr, res, it = kra.mc_trace(kra.DeviceMatrix(A, gpu_ctx), A.shape[0], 1e-12, 90, 0, seed=4, ctx=gpu_ctx)
    tro, reso, ito = ko.mc_trace(A, A.shape[0], 1e-12, 90, 0, seed=4)
    assert it == ito == 3
    assert tr == pytest.approx(tro, rel=1e-9, abs=1e-9)
    assert res == pytest.approx(reso, rel=1e-6, abs=1e-9)


def test_trace_exp_reference_composition(kra, gpu_ctx, values):
    """trace_exp.m with Afun = expmv (the reference composition)."""
    A = load_graph("oregon_A0")
    tr = kra.trace_exp(kra.DeviceMatrix(A, gpu_ctx), method="expmv", seed=1, ctx=gpu_ctx)
    tro = ko.trace_exp(A, seed=1)
    assert tr == pytest.approx(tro, rel=1e-9)
    assert tr == pytest.approx(values["oregon_A0"]["exact_tr_exp"], rel=1e-4)


def test_trace_exp_lanczos_config1(kra, gpu_ctx, values):
    """BASELINE.json configs[0]: dt_oregon A6 (n = 10,860), mc_trace + Lanczos
    (m = 20); one round = 30 probes; vs the oracle and the exact trace."""
    A = load_graph("oregon_A6")
    D = kra.DeviceMatrix(A, gpu_ctx)
    tr, res, it = kra.mc_trace("lanczos", A.shape[0], 1e-4, 30, 1, seed=0, m=20, A=D, ctx=gpu_ctx)
    tro, reso, ito = ko.trace_exp_lanczos(A, m=20, tol=1e-4, maxit=30, seed=0)
    assert it == ito == 1
    # measured 8.9e-14 (profiles/r01_config1.json); 1e-10 leaves room for the
    # Gauss-quadrature vs literal-vector forms (module docstring), not for drift
    assert tr == pytest.approx(tro, rel=1e-10)
    assert tr == pytest.approx(values["oregon_A6"]["exact_tr_exp"], rel=1e-3)
    full = kra.trace_exp(D, method="lanczos", m=20, seed=0, ctx=gpu_ctx)   # tol 1e-4, maxit 1000
    assert full == pytest.approx(values["oregon_A6"]["exact_tr_exp"], rel=1e-4)


@pytest.mark.parametrize("afun", ["expmv", "lanczos", "matrix"])
def test_mc_trace_twin_split_is_bit_identical(kra, gpu_ctx, monkeypatch, afun):
    """Each round's two quadratures (trace(Q' Afun Q) and trace(G' Afun G),
    mc_trace.m:46,49) run concurrently, the G term on the matrix's twin
    context: the same kernels on the same data as the serial order
    (KT_TWIN=0), so tr, res and the round count are bit-identical."""
    A = load_graph("oregon_A0")
    args = dict(n=A.shape[0], tol=1e-4, maxit=150, isAreal=1, seed=3, m=20)
    D = kra.DeviceMatrix(A, gpu_ctx)
    if afun == "matrix":
        par = kra.mc_trace(D, ctx=gpu_ctx, **args)
    else:
        par = kra.mc_trace(afun, A=D, ctx=gpu_ctx, **args)
    monkeypatch.setenv("KT_TWIN", "0")
    D2 = kra.DeviceMatrix(A, gpu_ctx)
    if afun == "matrix":
        ser = kra.mc_trace(D2, ctx=gpu_ctx, **args)
    else:
        ser = kra.mc_trace(afun, A=D2, ctx=gpu_ctx, **args)
    assert par == ser
    assert par[2] > 1  # several rounds (nested deflation) were run
    # the speculative next-round S term (third device copy, third thread) off:
    # still the same numbers
    monkeypatch.setenv("KT_TWIN", "1")
    monkeypatch.setenv("KT_MC_SPEC", "0")
    D3 = kra.DeviceMatrix(A, gpu_ctx)
    if afun == "matrix":
        nos = kra.mc_trace(D3, ctx=gpu_ctx, **args)
    else:
        nos = kra.mc_trace(afun, A=D3, ctx=gpu_ctx, **args)
    assert nos == par


def test_trace_exp_speculative_rounds_bit_identical(kra, gpu_ctx, monkeypatch):
    """trace_exp.m's composition (Afun = expmv, tol 1e-4, maxit 1000) with the
    next round's S term computed speculatively during the current round's Q
    and G terms (default) vs KT_MC_SPEC=0: the same estimate, bit for bit."""
    A = load_graph("oregon_A0")
    D = kra.DeviceMatrix(A, gpu_ctx)
    spec = kra.trace_exp(D, method="expmv", seed=2, ctx=gpu_ctx)
    monkeypatch.setenv("KT_MC_SPEC", "0")
    D2 = kra.DeviceMatrix(A, gpu_ctx)
    assert kra.trace_exp(D2, method="expmv", seed=2, ctx=gpu_ctx) == spec


@pytest.mark.parametrize("kind", ["loops", "signed"])
def test_expmv_normest1_branch_matches_oracle(kra, gpu_ctx, kind):
    """normAm.m:25-26: t (A - mu I) with negative entries (self loops after the
    shift, or signed weights) -> normest1 (t = 1) on the device (products and
    reductions on the device, the Higham-Tisseur iteration on the host); the
    same s, m, mv as the oracle's restatement and F to 1e-11."""
    from test_normest1 import looped, signed_graph
    A = looped(load_graph("oregon_A0")) if kind == "loops" else 4.0 * signed_graph(300, seed=5)
    b = np.random.default_rng(1).normal(size=(A.shape[0], 3))
    F, s, m, mv = kra.expmv(1.0, kra.DeviceMatrix(A, gpu_ctx), b, ctx=gpu_ctx)
    Fo, so, mo, mvo = ko.expmv(1.0, A, b)
    assert (s, m, mv) == (so, mo, mvo)
    np.testing.assert_allclose(F, Fo, rtol=1e-11, atol=1e-13 * np.abs(Fo).max())


def test_trace_exp_with_self_loops(kra, gpu_ctx):
    """trace_exp.m on a graph with self loops (expmv's shift mu != 0 and the
    normest1 branch): the oracle's estimate to 1e-9, the exact trace to 1e-4."""
    from test_normest1 import looped
    A = looped(load_graph("oregon_A0"))
    tr = kra.trace_exp(kra.DeviceMatrix(A, gpu_ctx), method="expmv", seed=1, ctx=gpu_ctx)
    assert tr == pytest.approx(ko.trace_exp(A, seed=1), rel=1e-9)
    exact = float(np.exp(np.linalg.eigvalsh(A.toarray())).sum())
    assert tr == pytest.approx(exact, rel=1e-4)


@pytest.mark.parametrize("name", ["oregon_A0", "rome", "oregon_A6"])
def test_mc_trace_batched_rounds_match_per_call(kra, gpu_ctx, monkeypatch, name):
    """The Lanczos-Afun mc_trace runs one probe sweep per round -- the round's
    Q and G terms and the next round's S term share a 30-column sweep
    (kt_mctrace.cpp mc_trace_batched) -- against the per-call form
    (KT_MC_BATCH=0, one sweep per Afun call): same probes and projections,
    only the sweep width differs, so the same rounds and the estimate to
    rounding (1e-11), over several rounds of nested deflation; and the
    oracle's numpy restatement of the same composition (1e-10)."""
    A = load_graph(name)
    D = kra.DeviceMatrix(A, gpu_ctx)
    args = dict(n=A.shape[0], tol=1e-8, maxit=150, isAreal=1, seed=5, m=20)
    b = kra.mc_trace("lanczos", A=D, ctx=gpu_ctx, **args)
    monkeypatch.setenv("KT_MC_BATCH", "0")
    p = kra.mc_trace("lanczos", A=D, ctx=gpu_ctx, **args)
    assert b[2] == p[2] and b[2] > 1
    assert b[0] == pytest.approx(p[0], rel=1e-11)
    if name != "oregon_A6":  # the numpy restatement at n = 10,860 x 5 rounds is slow
        tro, _, ito = ko.trace_exp_lanczos(A, m=20, tol=1e-8, maxit=150, seed=5)
        assert b[2] == ito and b[0] == pytest.approx(tro, rel=1e-10)


@pytest.mark.parametrize("name", ["oregon_A0", "rome"])
def test_mc_trace_next_s_term_guess_is_bit_identical(kra, gpu_ctx, monkeypatch, name):
    """The Lanczos-Afun mc_trace computes the next round's S term ahead unless
    the round is expected to stop (kt_mctrace.cpp mc_trace_batched); always
    ahead (KT_MC_AHEAD=1), never ahead (0) and the guess give the same round
    count and the estimate to rounding (a round with its S term ahead runs Q
    and G in explicit sweeps beside S, one without runs them by y-form
    sweeps: other reduction forms), over several rounds and a last round
    it == K (tol = 0)."""
    A = load_graph(name)
    D = kra.DeviceMatrix(A, gpu_ctx)
    for tol, maxit in ((1e-8, 150), (0.0, 90)):
        args = dict(n=A.shape[0], tol=tol, maxit=maxit, isAreal=1, seed=5, m=20)
        monkeypatch.delenv("KT_MC_AHEAD", raising=False)
        g = kra.mc_trace("lanczos", A=D, ctx=gpu_ctx, **args)
        monkeypatch.setenv("KT_MC_AHEAD", "1")
        a = kra.mc_trace("lanczos", A=D, ctx=gpu_ctx, **args)
        monkeypatch.setenv("KT_MC_AHEAD", "0")
        z = kra.mc_trace("lanczos", A=D, ctx=gpu_ctx, **args)
        assert g[2] == a[2] == z[2] and g[2] > 1
        assert a[0] == pytest.approx(g[0], rel=1e-12) and z[0] == pytest.approx(g[0], rel=1e-12)
        if tol == 0.0:
            assert g[2] == 3


def test_mc_trace_quadrature_columns_yform_vs_explicit(kra, gpu_ctx, monkeypatch):
    """The Q and G columns' forms by the y-form sweep (default) and by the
    explicit CGS2 sweep (KT_LC_YFORM=0) agree to rounding (a y-form column
    that trips the cancellation guard takes the explicit redo's records)."""
    A = load_graph("oregon_A6")
    D = kra.DeviceMatrix(A, gpu_ctx)
    args = dict(n=A.shape[0], tol=1e-8, maxit=150, isAreal=1, seed=2, m=20)
    y = kra.mc_trace("lanczos", A=D, ctx=gpu_ctx, **args)
    monkeypatch.setenv("KT_LC_YFORM", "0")
    x = kra.mc_trace("lanczos", A=D, ctx=gpu_ctx, **args)
    assert y[2] == x[2]
    assert y[0] == pytest.approx(x[0], rel=1e-11)
