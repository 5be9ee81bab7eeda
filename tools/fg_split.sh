#!/bin/bash
# Config 3 fun_and_grad: twin vs serial call time, and the host eigensolves of one call
# (KT_EIG_STATS=2 logs each: size, values/vectors, ms).
set -o pipefail
O=gpurun_out/fgs; mkdir -p $O
for tw in 1 0; do
  KT_TWIN=$tw timeout -k 10 120 python tools/prof_fg.py > $O/t$tw.txt 2>&1 || { tail -5 $O/t$tw.txt; exit 1; }
  echo "twin=$tw $(grep '^fg' $O/t$tw.txt | awk '{print $2}' | tr '\n' ' ')"
done
KT_EIG_STATS=2 timeout -k 10 120 python tools/prof_fg.py > $O/e.txt 2>&1 || { tail -5 $O/e.txt; exit 1; }
python3 - <<'PY'
import re
L = open("gpurun_out/fgs/e.txt").read().splitlines()
# the last fg call's eig lines: between the 3rd and 4th "fg" lines
idx = [i for i, l in enumerate(L) if l.startswith("fg ")]
seg = L[idx[2] + 1: idx[3]]
ev = [(int(m.group(1)), m.group(2), float(m.group(3))) for l in seg for m in [re.search(r"\[kt eig\] n (\d+) (\w+) ([\d.]+) ms", l)] if m]
print("eig calls in one fg:", len(ev), "total ms", round(sum(e[2] for e in ev), 2))
from collections import defaultdict
b = defaultdict(lambda: [0, 0.0])
for n, k, ms in ev:
    b[(k, (n // 25) * 25)][0] += 1; b[(k, (n // 25) * 25)][1] += ms
for key in sorted(b): print(key, b[key][0], round(b[key][1], 2))
print(L[idx[3]])
PY
