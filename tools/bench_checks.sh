# Bench checks: default line, --no-profile (event overhead), 2-rank rehearsal
# of the torchrun N>1 launch on one GPU (gloo sums, KT_BENCH_ONE_DEVICE=1).
set -o pipefail
O=gpurun_out/bchk; mkdir -p $O
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/b1.json 2> $O/b1.err || { tail $O/b1.err; exit 1; }
timeout -k 10 300 python bench.py --cpu-seconds 0 --no-profile > $O/b2.json 2> $O/b2.err || { tail $O/b2.err; exit 1; }
KT_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --dist-backend gloo > $O/b3.json 2> $O/b3.err || { tail $O/b3.err; exit 1; }
for f in b1 b2 b3; do python3 -c "import json,sys; d=json.loads([l for l in open('$O/$f.json') if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'], d['n_gpus'], d.get('roofline',{}).get('frac'))"; done
