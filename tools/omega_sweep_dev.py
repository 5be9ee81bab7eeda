"""Device fun_and_grad_krylov_fun over the Omega sweep fixture
(tests/golden/omega_sweep_values.json): per case the device objective's
distance to the exact value and to the oracle, and the gradient's."""
import json
import os
import sys

import torch  # noqa: F401
import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import krylov_robustness_amd as kra  # noqa: E402
from conftest import load_graph, GOLDEN  # noqa: E402

d = json.load(open(os.path.join(GOLDEN, "omega_sweep_values.json")))
A = load_graph("india")
ctx = kra.Context(0)
D = kra.DeviceMatrix(A, ctx)
for fun, c in d["cases"].items():
    for r in c["rows"]:
        f, gr = kra.fun_and_grad_krylov_fun(np.array(r["X"]), D, np.array(r["Omega"]), fun, c["dfun"],
                                            np.array(r["dfA"]), c["tol"], 100, ctx=ctx)
        gro = np.array(r["gr"])
        print(json.dumps({"fun": fun, "offset": r["offset"], "f": f, "dev_exact": abs(f - r["exact_f"]),
                          "oracle_exact": abs(r["f"] - r["exact_f"]), "dev_oracle": abs(f - r["f"]),
                          "gr_rel": float(np.abs(gr - gro).max() / np.abs(gro).max()),
                          "tol_f": c["tol_f"]}), flush=True)
