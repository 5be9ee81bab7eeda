set -e
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_qr.py tests/test_gpu_krylov.py tests/test_gpu_configs.py tests/test_gpu_omega_sweep.py tests/test_gpu_frechet.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do timeout -k 10 120 python tools/prof_fg.py > $O/fg$r.txt 2>&1; echo "fg: $(grep '^fg' $O/fg$r.txt | cut -c1-10 | tr '\n' ' ')"; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o k -- python3 tools/prof_fg.py > $O/prof.txt 2>&1
python3 - $(find $O/prof -name "*kernel_stats.csv") <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(f"{r['Name'][:44]:44s} {int(r['Calls']):6d} {int(r['TotalDurationNs'])/1e6:8.2f} ms avg {float(r['AverageNs'])/1e3:7.2f} us")
PY
