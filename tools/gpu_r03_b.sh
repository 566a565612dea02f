#!/bin/bash
# separate-launch breakdown of the cfg2 step (pipeline 0: draw, psort, grad, apply each alone)
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03b
mkdir -p $OUT
A="--no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 100 --warmup 10"
timeout -k 10 300 python bench.py $A --pipeline 0 > $OUT/p0.json 2> $OUT/p0.err || { echo "p0 failed"; tail -20 $OUT/p0.err; exit 1; }
timeout -k 10 300 python bench.py $A > $OUT/p1.json 2> $OUT/p1.err || { echo "p1 failed"; tail -20 $OUT/p1.err; exit 1; }
for f in p0 p1; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['ms_per_step'], {k:round(v['avg_us'],1) for k,v in d['kernels'].items() if k!='note'})"; done
