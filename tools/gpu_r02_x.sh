#!/bin/bash
# after the pos_sort owner fix: the 4-lane draw variant's pos_sort tests (it
# reproduced the race), the full check on the default build, then the draw
# group size timing A/B
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/x
B=collaborativefilteringusingtensorflow_amd/build
CF_ENGINE_LIB=$PWD/$B/variants/gl4/libcf_engine.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pos_sort.py -x -v --timeout 120 --timeout-method thread > gpurun_out/x/pytest_gl4.log 2>&1
rc=$?; echo "gl4 pos_sort tests: $(tail -1 gpurun_out/x/pytest_gl4.log)"; [ $rc -ne 0 ] && { grep -E "^E " gpurun_out/x/pytest_gl4.log | head -3; exit $rc; }
PYTEST_ARGS="-v --timeout 200 --timeout-method thread" bash tools/gpu_check.sh > gpurun_out/x/check.out 2>&1
rc=$?; tail -4 gpurun_out/x/check.out | cut -c1-300; [ $rc -ne 0 ] && exit $rc
cat > /tmp/psf.py <<'PY'
import sys, json
d = json.loads(sys.stdin.read()); k = d['kernels']
print(sys.argv[1], round(d['ms_per_step'], 4), {n: round(v['avg_us'], 1) for n, v in k.items() if n != 'note'})
PY
for r in 1 2; do
for v in default gl4; do
  lib=$PWD/$B/libcf_engine.so; [ $v != default ] && lib=$PWD/$B/variants/$v/libcf_engine.so
  CF_ENGINE_LIB=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 >> gpurun_out/x/cfg2_$v.jsonl 2>> gpurun_out/x/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/x/bench.err; exit 1; }
  tail -1 gpurun_out/x/cfg2_$v.jsonl | python /tmp/psf.py "cfg2 $v"
done
done
