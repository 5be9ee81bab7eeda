# deferred profiling-event collection: bench with and without the per-launch events, bench tests, slq tests
set -e
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 300 python bench.py --steps 5 --cpu-seconds 0 > $O/prof.json 2>$O/prof.err
timeout -k 10 300 python bench.py --steps 5 --cpu-seconds 0 --no-profile > $O/noprof.json 2>/dev/null
timeout -k 10 300 python bench.py --steps 5 --cpu-seconds 0 > $O/prof2.json 2>>$O/prof.err
python3 - <<'PY'
import json
for f in ("prof", "noprof", "prof2"):
    d = json.load(open(f"gpurun_out/r03i/{f}.json"))
    r = d.get("roofline") or {}
    print(f, d["value"], "evals/s", "avg_launch_us", r.get("avg_launch_us"), "iso", (r.get("isolated_pass") or {}).get("avg_launch_us"), "frac", r.get("frac"))
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_slq.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
