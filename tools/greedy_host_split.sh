# Config 5: whole-run time vs the fused candidate launches (KT_PAIRS_TIMING)
set -o pipefail
O=gpurun_out/ghs; mkdir -p $O
KT_PAIRS_TIMING=1 timeout -k 10 120 python tests/perf/bench_greedy.py --cpu-steps 0 --repeat 1 > $O/b.json 2> $O/err.txt || { tail $O/err.txt; exit 1; }
cut -c1-200 $O/b.json
grep "fused C=" $O/err.txt | tail -50 | awk '{s+=$(NF-1)} END {print "last 50 batches gpu ms:", s}'
