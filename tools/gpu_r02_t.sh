#!/bin/bash
# the default bench line (CPU baselines, NDCG), a 2-rank gloo rehearsal of
# bench.py --gpus 2 (self-launched, ranks sharing device 0), cfg3 / cfg4 / cfg5
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/final
timeout -k 10 400 python bench.py > gpurun_out/final/cfg2.json 2> gpurun_out/final/cfg2.err || { echo "bench failed"; tail -20 gpurun_out/final/cfg2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/final/cfg2.json')); print('cfg2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['batch_65536']['value'], d['cpu_baseline']['value'])"
CF_DIST_BACKEND=gloo CF_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 50 --warmup 5 --secondary-batch 0 > gpurun_out/final/dist2_gloo.json 2> gpurun_out/final/dist2_gloo.err || { echo "dist2 failed"; tail -20 gpurun_out/final/dist2_gloo.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/final/dist2_gloo.json')); print('dist2', d['n_gpus'], d['value'], d['config']['world_size_formed'], d['config']['backend'], d['kernels'].get('psort'))"
for c in cfg3 cfg4 cfg5; do
  timeout -k 10 500 python bench.py --config $c --no-cpu-baseline --no-ndcg > gpurun_out/final/$c.json 2> gpurun_out/final/$c.err || { echo "$c failed"; tail -20 gpurun_out/final/$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/final/$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], {n: round(v['avg_us'],1) for n,v in d['kernels'].items() if n!='note'})"
done
