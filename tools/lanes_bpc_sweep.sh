# headline: sweep lanes x workgroups-per-CU of the y-form pass (bench, 5 steps, no CPU baseline)
set -e
O=gpurun_out/lbpc; mkdir -p $O
for l in 2 3; do for b in 3 4 6; do
  KT_KY_BPC=$b timeout -k 10 300 python bench.py --lanes $l --steps 5 --cpu-seconds 0 --no-profile > $O/l${l}_b${b}.json 2>/dev/null
  python3 -c "import json; d=json.load(open('$O/l${l}_b${b}.json')); print('lanes $l bpc $b', d['value'], 'evals/s')"
done; done
KT_KY_BPC=4 timeout -k 10 300 python bench.py --lanes 2 --steps 5 --cpu-seconds 0 --no-profile > $O/l2_b4_again.json 2>/dev/null
python3 -c "import json; d=json.load(open('$O/l2_b4_again.json')); print('lanes 2 bpc 4 (again)', d['value'], 'evals/s')"
