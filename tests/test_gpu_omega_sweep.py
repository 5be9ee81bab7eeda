"""fun_and_grad_krylov_fun over a fixed sweep of Omega, not a hand-picked one
(tests/golden/make_omega_sweep.py -> omega_sweep_values.json): voltage India,
Omega = 5 consecutive upper edges at offsets 0, 5, ..., 95, (sinh, cosh) and
(cosh, sinh), tol = 1e-6 f(normest(A, 1e-2)), it = 100
(Tests/test_weighted_sinh_lbfgs.m / _cosh_ settings; fun_and_grad_krylov_fun.m).

Tolerance rule (stated once, applied to every case):
  * gradient (fun_update's full-basis block Arnoldi, fun_update.m): 1e-8
    relative to the oracle (measured <= 2e-10);
  * objective (trace_fun_update's 2-block window, trace_fun_update.m): either
    the device agrees with the oracle to rounding, |f - f_o| <= 1e-9 max(|f_o|,
    tol_f), or -- where the 25-column power-grid block is numerically rank
    deficient and qr(w, 0)'s rounding-dependent completion direction enters
     -- the device is no further from the exact objective than
    the reference algorithm's own error or its stopping tolerance:
    |f - f_exact| <= max(tol_f, |f_o - f_exact|), with tol_f = tol f(normest)
    the tolerance fun_and_grad_krylov_fun.m:65 hands to trace_fun_update and
    f_exact from dense eigvalsh.  At least 38 of the 40 cases must take the
    first branch: the measured count, offset 60 taking the second for both
    funs (the slack of two cases that round 3 allowed is gone).
The sweep also shows the reference algorithm's own inaccuracy: the oracle is
further than tol_f from the exact objective in 4 of the 40 cases."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_graph

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sweep():
    with open(os.path.join(GOLDEN, "omega_sweep_values.json")) as f:
        return json.load(f)


def test_fun_and_grad_fun_omega_sweep(gpu_ctx, sweep):
    import krylov_robustness_amd as kra
    A = load_graph("india")
    D = kra.DeviceMatrix(A, gpu_ctx)
    assert kra.normest(D, 1e-2, ctx=gpu_ctx) == pytest.approx(sweep["normest_1e-2"], rel=1e-12)
    rounding, report = 0, []
    for fun, case in sweep["cases"].items():
        tol_f = case["tol_f"]
        for r in case["rows"]:
            f, gr = kra.fun_and_grad_krylov_fun(np.array(r["X"]), D, np.array(r["Omega"], dtype=np.int64),
                                                fun, case["dfun"], np.array(r["dfA"]), case["tol"], 100,
                                                ctx=gpu_ctx)
            gro = np.array(r["gr"])
            np.testing.assert_allclose(gr, gro, rtol=1e-8, atol=1e-8 * np.abs(gro).max(),
                                       err_msg=f"{fun} offset {r['offset']}")
            f_o, f_x = r["f"], r["exact_f"]
            if abs(f - f_o) <= 1e-9 * max(abs(f_o), tol_f):
                rounding += 1
            else:
                report.append((fun, r["offset"], abs(f - f_o), abs(f - f_x), abs(f_o - f_x)))
                assert abs(f - f_x) <= max(tol_f, abs(f_o - f_x)), (fun, r["offset"], f, f_o, f_x)
    assert rounding >= 38, report
