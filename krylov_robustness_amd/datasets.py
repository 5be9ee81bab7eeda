"""Loading the reference's graph datasets the way its drivers do
(SURVEY.md §8f row 4).

``load_problem(path)`` reads ``Problem.A`` (or any top-level variable) from a
MAT-file of either flavour the reference ships: MAT v5 through scipy.io, MAT
v7.3 (HDF5: datasets_paper/Misc/CollegeMsg.mat, Drugs.mat, as_735.mat)
through the package's own reader (matv73.py; h5py is absent).

``prepare_unweighted`` is the preprocessing of the unweighted drivers,
test_unweighted_make.m:41-52 / test_unweighted_break.m:42-52:

    A = Problem.A;
    A = spones(A + A');                       % symmetric, unit weights
    A = A - spdiags(diag(A), 0, n, n);        % no self loops
    ind = max_connected_component(A); A = A(ind, ind);

(max_connected_component is the drivers' local function,
Tests/test_unweighted_make.m:159-168: conncomp bins numbered in discovery
order from node 1, the first largest bin kept -- scipy labels components in
the same order, and argmax keeps the first maximum).  ``prepare_weighted``
is test_weighted_exp_lbfgs.m:34-36 (A / max(A(:))).  Host-side input
preparation only: the result is handed to DeviceMatrix.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.csgraph as csg

from . import matv73

_HDF5_SIG = b"\x89HDF\r\n\x1a\n"


def is_v73(path) -> bool:
    with open(path, "rb") as f:
        head = f.read(520)
    return head[:8] == _HDF5_SIG or head[512:520] == _HDF5_SIG


def load_variable(path, name="Problem"):
    """Top-level variable `name` of a MAT-file (v5 or v7.3).  Structs come
    back as dicts in both cases."""
    if is_v73(path):
        return matv73.loadmat(path, variables=[name])[name]
    import scipy.io as sio
    v = sio.loadmat(path, variable_names=[name])[name]
    if v.dtype.names:  # 1x1 struct -> dict
        return {k: v[k][0, 0] for k in v.dtype.names}
    return v


def load_problem(path, field="A"):
    """Problem.A of a SuiteSparse-style MAT-file, as CSR float64."""
    P = load_variable(path, "Problem")
    return sp.csr_matrix(P[field], dtype=np.float64)


def max_connected_component(A):
    """Indices of the largest connected component of the (symmetric)
    pattern of A, ascending."""
    _, lab = csg.connected_components(sp.csr_matrix(A), directed=False)
    big = np.argmax(np.bincount(lab))
    return np.flatnonzero(lab == big)


def prepare_unweighted(A):
    """spones(A + A'), diagonal removed, largest connected component."""
    A = sp.csr_matrix(A, dtype=np.float64)
    A = ((A + A.T) != 0).astype(np.float64).tocsr()
    A.setdiag(0)
    A.eliminate_zeros()
    ind = max_connected_component(A)
    A = A[ind][:, ind].tocsr()
    A.sort_indices()
    return A


def prepare_weighted(A):
    """A / max(A(:))  (test_weighted_exp_lbfgs.m:34-36)."""
    A = sp.csr_matrix(A, dtype=np.float64)
    return (A / A.max()).tocsr()


def load_unweighted(path):
    """load + prepare, exactly the unweighted drivers' sequence."""
    return prepare_unweighted(load_problem(path))
