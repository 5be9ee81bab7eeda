"""Exact spectrum identities for config 3's graph (Hawaii LCC, n = 21,774):
tr(sinh(A)), tr(cosh(A)), tr(exp(A)) and the squared Frobenius norms
sum f(lambda)^2 (the bound 2 ||f(A)||_F^2 / N on a Rademacher Hutchinson
estimate's variance) from a dense eigvalsh (a few minutes, a ~4 GB matrix)
-> hawaii_values.json.  Build container only."""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from conftest import load_graph  # noqa: E402

t = time.time()
A = load_graph("hawaii")
d = np.linalg.eigvalsh(A.toarray())
rec = {"n": int(A.shape[0]), "nnz": int(A.nnz), "lambda_max": float(d.max()),
       "exact_tr_exp": float(np.sum(np.exp(d))), "exact_tr_sinh": float(np.sum(np.sinh(d))),
       "exact_tr_cosh": float(np.sum(np.cosh(d))),
       "frob2_sinh": float(np.sum(np.sinh(d) ** 2)), "frob2_cosh": float(np.sum(np.cosh(d) ** 2)),
       "frob2_exp": float(np.sum(np.exp(d) ** 2)), "seconds": time.time() - t}
with open(os.path.join(HERE, "hawaii_values.json"), "w") as f:
    json.dump(rec, f, indent=1)
print(rec)
