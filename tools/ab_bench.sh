#!/bin/bash
# A/B of hot-path variants on ONE box (same GPU, back to back).  Each line:
#   label|ENV=VAL ENV2=VAL2|extra bench args
# Usage (GPU box, repo root): bash tools/ab_bench.sh TAG VARIANTS_FILE
set -o pipefail
TAG=${1:-ab}; VF=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
: > $OUT/ab.txt
while IFS='|' read -r label envs args; do
    [ -z "$label" ] && continue
    case "$label" in \#*) continue;; esac
    line=$(env $envs timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 $args 2> $OUT/$label.err) || { echo "$label FAILED"; tail -5 $OUT/$label.err; exit 1; }
    echo "$line" > $OUT/$label.json
    python3 - "$label" "$envs" "$args" "$line" >> $OUT/ab.txt <<'PY'
import json, sys
label, envs, args, line = sys.argv[1:5]
b = json.loads(line)
r = b.get("roofline") or {}
print(f"{label:22s} {b['value']:.4f} evals/s  {b['ms_per_step']:8.2f} ms/eval  iso pass {r.get('avg_launch_us')} us  "
      f"overlapped {r.get('timed_region_avg_launch_us_overlapped')} us  [{envs} {args}]")
PY
    tail -1 $OUT/ab.txt
done < $VF
