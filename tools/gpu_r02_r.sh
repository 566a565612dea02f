#!/bin/bash
# pos_sort 16-B records: its parity tests + the step parity suite, the A/B at
# 2^19, then the rocprof trace + PMC passes of the default line
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/psort4
timeout -k 10 600 python -u -m pytest tests/test_gpu_pos_sort.py tests/test_gpu_step_parity.py tests/test_gpu_pipeline.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > gpurun_out/psort4/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/psort4/pytest.log; [ $rc -ne 0 ] && { echo "PYTEST rc=$rc"; exit $rc; }
for v in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 --pos-sort $v >> gpurun_out/psort4/ab.jsonl 2>> gpurun_out/psort4/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/psort4/bench.err; exit 1; }
  tail -1 gpurun_out/psort4/ab.jsonl | python -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print('pos_sort=$v', round(d['ms_per_step'],4), {n: round(v['avg_us'],1) for n,v in k.items() if n!='note'})"
done
TAG=cfg2_b524288 BENCH_ARGS="--steps 100 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0" bash tools/gpu_profile.sh > /dev/null || exit 1
echo done
