#!/bin/bash
# one-launch psort: pos_sort + distributed tests (both sort forms), then the
# A/B psort_fused 1 vs 0 at cfg2 and the rocprof trace of the default line
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/psort6
timeout -k 10 600 python -u -m pytest tests/test_gpu_pos_sort.py tests/test_gpu_distributed.py -x -v --timeout 200 --timeout-method thread > gpurun_out/psort6/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/psort6/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/psort6/pytest.log | head; echo "PYTEST rc=$rc"; exit $rc; }
cat > /tmp/psf.py <<'PY'
import sys, json
d = json.loads(sys.stdin.read()); k = d['kernels']
print(sys.argv[1], round(d['ms_per_step'], 4), {n: round(v['avg_us'], 1) for n, v in k.items() if n != 'note'})
PY
for v in 1 0 1 0; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 >> gpurun_out/psort6/ab.jsonl 2>> gpurun_out/psort6/bench.err --psort-fused $v || { echo "BENCH FAILED"; tail -20 gpurun_out/psort6/bench.err; exit 1; }
  tail -1 gpurun_out/psort6/ab.jsonl | python /tmp/psf.py "psort_fused=$v"
done
TAG=cfg2_b524288 BENCH_ARGS="--steps 100 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0" bash tools/gpu_profile.sh > /dev/null || exit 1
echo done
