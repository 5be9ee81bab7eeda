"""A/B on one GPU box: CGS2 Gram blocks kept on the device (default) vs the
host round trip per pass (KT_GRAM_HOST=1), alternating runs of the hessian
and config-3 benches; prints one JSON line per variant with the best times."""
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))


def run(tool, env, *args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "perf", tool), *args], env=env,
                         capture_output=True, text=True, timeout=300, check=True).stdout
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


best = {}
for rep in range(2):
    for v in ("0", "1"):
        env = dict(os.environ, KT_GRAM_HOST=v)
        h = run("bench_hessian.py", env)
        c = run("bench_config3.py", env, "--no-oracle")
        b = best.setdefault(v, {})
        for k, val in (("fg_exp_s", h["fg_s"]), ("hessian_s", h["hessian_s"]), ("fg_fun_s", c["fg_s"]),
                       ("fme_s", c["fme_s"])):
            b[k] = min(b.get(k, 1e9), val)
        b["fg_fun_f"] = c["fg_f"]
for v, b in best.items():
    print(json.dumps({"KT_GRAM_HOST": v, **b}))
