#!/bin/bash
# Round-3 final pass, part 2: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE
# passes and the bench line of cfg2..cfg5 on the committed build
# (tools/gpu_profile_cfg.sh), then the 2-rank gloo rehearsal of the sharded line.
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03final2
mkdir -p $OUT
for c in cfg3 cfg5 cfg4; do
  bash tools/gpu_profile_cfg.sh r03g_$c --config $c || exit 1
done
CF_DIST_BACKEND=gloo CF_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 \
  --no-cpu-baseline --no-ndcg --secondary-batch 0 > $OUT/dist2_gloo.json 2> $OUT/dist2_gloo.err || { echo "gloo rehearsal failed"; tail -20 $OUT/dist2_gloo.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/dist2_gloo.json').read().strip().splitlines()[-1]); r=d['roofline']; print('dist2', d['n_gpus'], d['value'], 'frac', r['frac'], 'traffic', r['traffic'], r['pmc_key'])"
