#!/bin/bash
# draw group size A/B: 8 lanes per pair (default) against 4 (16 chunks in
# flight) and 2 (32): sampler / pipeline GPU tests on each variant, then the
# cfg2 line alternating, and cfg4 (GBPR) once each
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/gl
B=collaborativefilteringusingtensorflow_amd/build
for v in; do
  CF_ENGINE_LIB=$PWD/$B/variants/$v/libcf_engine.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_pipeline.py tests/test_gpu_pos_sort.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gl/pytest_$v.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/gl/pytest_$v.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/gl/pytest_$v.log | head -5; exit $rc; }
done
cat > /tmp/psf.py <<'PY'
import sys, json
d = json.loads(sys.stdin.read()); k = d['kernels']
print(sys.argv[1], round(d['ms_per_step'], 4), {n: round(v['avg_us'], 1) for n, v in k.items() if n != 'note'})
PY
for r in 1 2; do
for v in default gl4 gl2; do
  lib=$PWD/$B/libcf_engine.so; [ $v != default ] && lib=$PWD/$B/variants/$v/libcf_engine.so
  CF_ENGINE_LIB=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 >> gpurun_out/gl/cfg2_$v.jsonl 2>> gpurun_out/gl/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/gl/bench.err; exit 1; }
  tail -1 gpurun_out/gl/cfg2_$v.jsonl | python /tmp/psf.py "cfg2 $v"
done
done
for v in default gl4 gl2; do
  lib=$PWD/$B/libcf_engine.so; [ $v != default ] && lib=$PWD/$B/variants/$v/libcf_engine.so
  CF_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --config cfg4 --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 >> gpurun_out/gl/cfg4_$v.jsonl 2>> gpurun_out/gl/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/gl/bench.err; exit 1; }
  tail -1 gpurun_out/gl/cfg4_$v.jsonl | python /tmp/psf.py "cfg4 $v"
done
