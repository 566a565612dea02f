#!/bin/bash
# final build: a 4-rank gloo rehearsal of bench --gpus 4 (ranks sharing device
# 0; exercises the sharded step with pos_sort in the item reduce), cfg3 / cfg4 / cfg5 lines
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/y
CF_DIST_BACKEND=gloo CF_SHARE_DEVICE=1 timeout -k 10 500 python bench.py --gpus 4 --steps 30 --warmup 3 --secondary-batch 0 --no-profile > gpurun_out/y/dist4_gloo.json 2> gpurun_out/y/dist4_gloo.err || { echo "dist4 failed"; tail -20 gpurun_out/y/dist4_gloo.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/y/dist4_gloo.json')); print('dist4', d['n_gpus'], d['config']['world_size_formed'], d['config']['backend'], d['config']['item_exchange'], d['value'])"
for c in cfg3 cfg4 cfg5; do
  timeout -k 10 500 python bench.py --config $c --no-cpu-baseline --no-ndcg > gpurun_out/y/$c.json 2> gpurun_out/y/$c.err || { echo "$c failed"; tail -20 gpurun_out/y/$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/y/$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
