#!/bin/bash
# Config 2 (Erdos-Renyi n = 100k, 128 probes x m = 30): probe block P x sweep lanes, y-form pass.
set -o pipefail
O=gpurun_out/er; mkdir -p $O
for P in 128 64 32 16; do
  for L in 1 2 4; do
    timeout -k 10 120 python bench.py --config er100k --steps 20 --warmup 3 --cpu-seconds 0 --block $P --lanes $L > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print('P=$P lanes=$L', d['value'], 'evals/s', d['ms_per_step'], 'ms', 'pass', r.get('avg_launch_us'), 'iso', (r.get('isolated_pass') or {}).get('avg_launch_us'))"
  done
done
