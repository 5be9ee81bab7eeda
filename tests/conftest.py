import json
import os
import sys

# Load torch (and its bundled ROCm runtime / rocBLAS / rocSOLVER) BEFORE
# libkrylov_hip.so: the library's NEEDED entries (libamdhip64.so.7,
# librocblas.so.5, librocsolver.so.0) then bind to the copies torch already
# mapped, so one process never holds two ROCm runtimes.  bench.py does the same.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

import numpy as np
import pytest
import scipy.sparse as sp

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun)")


def load_graph(name):
    z = np.load(os.path.join(GOLDEN, "hawaii.npz" if name == "hawaii" else "graphs.npz"))
    n = int(z[name + "__n"][0])
    return sp.csr_matrix((z[name + "__data"], z[name + "__indices"], z[name + "__indptr"]),
                         shape=(n, n))


def load_v73_graph(name):
    """A prepared MAT v7.3 dataset (drugs / as_735 / collegemsg), make_golden.py --v73."""
    z = np.load(os.path.join(GOLDEN, "v73_graphs.npz"))
    n = int(z[name + "__n"][0])
    return sp.csr_matrix((z[name + "__data"], z[name + "__indices"], z[name + "__indptr"]),
                         shape=(n, n))


def golden_values():
    with open(os.path.join(GOLDEN, "values.json")) as f:
        return json.load(f)


GRAPHS = ["oregon_A0", "anaheim", "rome", "denmark", "austria", "india"]


@pytest.fixture(scope="session")
def values():
    return golden_values()


@pytest.fixture(scope="session")
def gpu_ctx():
    import krylov_robustness_amd as kra
    return kra.Context(0)


def iter_matches(it_dev, it_oracle, hist, tol, rel=1e-11):
    """Iteration counts of a lag-2 stop test (trace_fun_update.m:104-118) agree
    exactly, or differ by one step where the oracle's decision at that step was
    marginal: |err - tol| <= rel max(|Xm|, tol), the band that the device's
    rounding-level difference in Xm (measured <= 1e-12 relative on these
    graphs) can move err across.
    hist: the oracle's [(j, err, Xm), ...] (krylov_oracle.trace_fun_update)."""
    it_dev, it_oracle = int(it_dev), int(it_oracle)
    if it_dev == it_oracle:
        return True
    if abs(it_dev - it_oracle) != 1:
        return False
    j = min(it_dev, it_oracle)  # one side stopped here, the other did not
    for jj, err, xm in hist:
        if jj == j:
            return abs(err - tol) <= rel * max(abs(xm), tol)
    return False
