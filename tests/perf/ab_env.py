"""A/B of one environment switch on one GPU box: alternating runs of the
block-Krylov / greedy / config-1 benches with VAR=a and VAR=b; best times.
  python tests/perf/ab_env.py VAR a b"""
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
var, vals = sys.argv[1], sys.argv[2:4]


def run(tool, env, *args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "perf", tool), *args], env=env,
                         capture_output=True, text=True, timeout=300, check=True).stdout
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


best = {}
for rep in range(2):
    for v in vals:
        env = dict(os.environ, **{var: v})
        h = run("bench_hessian.py", env)
        c = run("bench_config3.py", env, "--no-oracle")
        g = run("bench_greedy.py", env)
        b = best.setdefault(v, {})
        for k, val in (("fg_exp_s", h["fg_s"]), ("hessian_s", h["hessian_s"]), ("fg_fun_s", c["fg_s"]),
                       ("fme_s", c["fme_s"]), ("greedy_s", g["gpu_seconds"])):
            b[k] = min(b.get(k, 1e9), val)
        b["fg_fun_f"], b["greedy_rob"] = c["fg_f"], g["rob_variation"]
for v, b in best.items():
    print(json.dumps({var: v, **b}))
