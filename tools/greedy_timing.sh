KT_PAIRS_TIMING=1 timeout -k 10 200 python tests/perf/bench_greedy.py --cpu-steps 0 --repeat 1 > gpurun_out/gt.json 2> gpurun_out/gt.err; python3 - <<'PY'
import re
L = open("gpurun_out/gt.err").read().splitlines()
def avg(pat):
    v = [float(m.group(1)) for l in L for m in [re.search(pat, l)] if m]
    return (len(v), sum(v) / len(v) if v else 0)
print("natural CSR", avg(r"natural CSR ([0-9.]+) ms"))
print("fused (prep+kernel+sync)", avg(r"fused C=\d+ n=\d+ ([0-9.]+) ms"))
print("score", avg(r"score ([0-9.]+) ms"))
print("select+edit", avg(r"select\+edit ([0-9.]+) ms"))
PY
