#!/bin/bash
# vectorised row scan in the draw + grad_sort_kernel: sampler / pos_sort parity,
# then same-box A/B prep1 (scalar draw) / default (16-B row loads) / sortw8 (+ SORT kernel at <= 64 VGPRs)
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03h
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_pos_sort.py tests/test_gpu_models.py \
  tests/test_gpu_pipeline.py -m gpu -q -rf -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && { echo "pytest rc $rc"; exit $rc; }
B=collaborativefilteringusingtensorflow_amd/build
A="--no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 200 --warmup 20"
cat > /tmp/psf.py <<'PY'
import sys, json
d = json.loads(sys.stdin.read()); k = d['kernels']
print(sys.argv[1], round(d['ms_per_step'], 4), {n: round(v['avg_us'], 1) for n, v in k.items() if n != 'note'})
PY
for r in 1 2; do
for v in prep1 default sortw8; do
  lib=$PWD/$B/libcf_engine.so; [ $v != default ] && lib=$PWD/$B/variants/$v/libcf_engine.so
  CF_ENGINE_LIB=$lib timeout -k 10 200 python bench.py $A >> $OUT/cfg2_$v.jsonl 2>> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
  tail -1 $OUT/cfg2_$v.jsonl | python /tmp/psf.py "cfg2 $v"
done
done
