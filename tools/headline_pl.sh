#!/bin/bash
# Headline: probe block x lanes re-check with the round-2 pass (16 B per lane).
set -o pipefail
O=gpurun_out/hpl; mkdir -p $O
for cfg in "16 2" "32 1" "32 2" "16 3" "8 4"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --block $1 --lanes $2 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); r=d['roofline'] or {}; print('P=$1 lanes=$2', d['value'], 'evals/s', d['ms_per_step'], 'ms', 'pass', r.get('avg_launch_us'), 'iso', (r.get('isolated_pass') or {}).get('avg_launch_us'))"
done
