#!/bin/bash
# compact negative slots + dense pos_sort apply: parity of every pos_sort path, then the cfg2 line
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pos_sort.py tests/test_gpu_models.py tests/test_gpu_distributed.py \
  -m gpu -q -rf -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
[ $rc -ne 0 ] && { echo "pytest rc $rc"; exit $rc; }
A="--no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 100 --warmup 10"
timeout -k 10 300 python bench.py $A > $OUT/p1.json 2> $OUT/p1.err || { echo "p1 failed"; tail -20 $OUT/p1.err; exit 1; }
timeout -k 10 300 python bench.py $A --pipeline 0 > $OUT/p0.json 2> $OUT/p0.err || { echo "p0 failed"; tail -20 $OUT/p0.err; exit 1; }
for f in p1 p0; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['ms_per_step'], d['roofline']['frac'], {k:round(v['avg_us'],1) for k,v in d['kernels'].items() if k!='note'})"; done
