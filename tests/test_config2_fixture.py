"""BASELINE config 2's reference value (tests/golden/config2_values.json,
written by tests/golden/make_config2_fixture.py), checked on the CPU.

The fixture's tr(exp A) of the Erdos-Renyi bench graph is the sum of all n
diagonal entries e_i' exp(A) e_i, each by m = 30 Lanczos steps from e_i +
Gauss quadrature (no sampling error).  Here: that per-row method agrees with
SciPy's expm_multiply (Al-Mohy & Higham, an independent algorithm) to 1e-13
on sample rows (the highest degree included); the fixture's forms are the C
oracle's; and every Hutchinson estimate the fixture holds (5 x 128 probes,
8,192 probes) lies within 3 true standard errors of the diagonal sum, the
standard error from the fixture's exact variance 2 (||exp A||_F^2 -
sum exp(A)_ii^2) per probe."""
import json
import math
import os

import numpy as np
import pytest

from conftest import ROOT
from oracle import slq_ref

FIX = os.path.join(ROOT, "tests", "golden", "config2_values.json")


@pytest.fixture(scope="module")
def fx():
    with open(FIX) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def A():
    from krylov_robustness_amd import graphs
    return graphs.erdos_renyi(100_000, 500_000, seed=0).tocsr()


def test_graph_matches_fixture(fx, A):
    assert (A.shape[0], A.nnz) == (fx["n"], fx["nnz"])


def test_unit_vector_quadrature_matches_expm_multiply(A):
    import scipy.sparse.linalg as sla
    deg = np.diff(A.indptr)
    rows = [0, 4242, 99_999, int(np.argmax(deg)), int(np.argmin(deg))]
    for i in rows:
        e = np.zeros(A.shape[0])
        e[i] = 1.0
        ref = sla.expm_multiply(A, e)[i]
        q = slq_ref.unit_quad(A, i, 1, 30, (1.0, 2.0))[0]
        assert q[0] == pytest.approx(ref, rel=1e-13)
        assert q[1] == pytest.approx(float(np.dot(sla.expm_multiply(A, e), sla.expm_multiply(A, e))), rel=1e-12)


def test_fixture_forms_are_the_c_oracles(fx, A):
    q = np.array(fx["slq_exp"]["seeds"]["0"]["q"])
    _, q_ref = slq_ref.slq_trace(A, 3, 30, seed=0)
    np.testing.assert_allclose(q_ref, q[:3], rtol=1e-13)
    _, q_ref = slq_ref.slq_trace(A, 2, 30, seed=4, probe_offset=126)
    np.testing.assert_allclose(q_ref, fx["slq_exp"]["seeds"]["4"]["q"][126:], rtol=1e-13)


def test_hutchinson_estimates_within_true_stderr(fx):
    ex = fx["exact"]
    tr, var1 = ex["tr_exp"], ex["hutchinson_var_per_probe"]
    assert ex["m45_max_rel_diff"] < 1e-12  # the quadrature has converged at m = 30
    assert 0 < ex["sum_diag_sq"] < ex["fro2_exp"]
    se128 = math.sqrt(var1 / 128)
    ests = [v["estimate"] for v in fx["slq_exp"]["seeds"].values()]
    for e in ests:
        assert abs(e - tr) <= 3 * se128
    assert abs(np.mean(ests) - tr) <= 3 * se128 / math.sqrt(len(ests))
    h = fx["hutchinson_8192"]
    assert abs(h["estimate"] - tr) <= 3 * math.sqrt(var1 / 8192)
    # the sample standard errors estimate the true one
    assert h["sample_stderr"] == pytest.approx(h["true_stderr"], rel=0.1)
