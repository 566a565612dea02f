#!/bin/bash
# full check (smoke, every GPU test, default bench line), then the pos_sort
# A/B at 2^19 and the rocprof trace + PMC passes of the default line
set -o pipefail
export PYTHONUNBUFFERED=1
PYTEST_ARGS="-v --timeout 120 --timeout-method thread" bash tools/gpu_check.sh > gpurun_out/check.out 2>&1
rc=$?; tail -8 gpurun_out/check.out | cut -c1-300; [ $rc -ne 0 ] && { echo "CHECK rc=$rc"; exit $rc; }
mkdir -p gpurun_out/psort3
for v in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 --pos-sort $v >> gpurun_out/psort3/ab.jsonl 2>> gpurun_out/psort3/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/psort3/bench.err; exit 1; }
  tail -1 gpurun_out/psort3/ab.jsonl | python -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print('pos_sort=$v', round(d['ms_per_step'],4), {n: round(v['avg_us'],1) for n,v in k.items() if n!='note'})"
done
TAG=cfg2_b524288 BENCH_ARGS="--steps 100 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0" bash tools/gpu_profile.sh > /dev/null || exit 1
echo done
