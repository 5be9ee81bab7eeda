# Headline y-form pass: probes per sweep (P) x sweep lanes, default command otherwise
# (bench.py, no profiler, no CPU leg); one bench process per setting, alternating twice.
set -e
O=$PWD/gpurun_out/blk; mkdir -p $O
for rep in 1 2; do
  for cfg in "16 2" "32 1" "32 2" "16 3"; do
    set -- $cfg
    timeout -k 10 120 python bench.py --steps 4 --warmup 1 --block $1 --lanes $2 --cpu-seconds 0 --no-profile > $O/b$1_l$2_r$rep.json 2> $O/b$1_l$2_r$rep.err
    python3 -c "import json,sys;d=json.loads(open('$O/b$1_l$2_r$rep.json').read().strip().splitlines()[-1]);print('P',$1,'lanes',$2,'rep',$rep,d['value'],'evals/s',d['ms_per_step'],'ms/step')"
  done
done
