#!/bin/bash
# pos_sort: its GPU parity tests, the fold-replica oracle test, then a cfg2 /
# cfg5 A/B of the option on one box (JSON lines under gpurun_out/psort/)
set -o pipefail
mkdir -p gpurun_out/psort
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pos_sort.py "tests/test_gpu_models.py::test_fold_parallel_replicas_match_oracle" -x -v --timeout 120 --timeout-method thread > gpurun_out/psort/pytest.log 2>&1
rc=$?
tail -12 gpurun_out/psort/pytest.log
if [ $rc -ne 0 ]; then echo "PYTEST rc=$rc"; exit $rc; fi
for v in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 --pos-sort $v >> gpurun_out/psort/cfg2.jsonl 2>> gpurun_out/psort/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/psort/bench.err; exit 1; }
  tail -1 gpurun_out/psort/cfg2.jsonl | python -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print('cfg2 pos_sort=$v', round(d['ms_per_step'],4), {n: round(v['avg_us'],1) for n,v in k.items() if n!='note'})"
done
for v in "--item-slots 1 --pos-sort 0" "--item-slots 0 --pos-sort 1"; do
  timeout -k 10 200 python bench.py --config cfg5 --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 $v >> gpurun_out/psort/cfg5.jsonl 2>> gpurun_out/psort/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/psort/bench.err; exit 1; }
  tail -1 gpurun_out/psort/cfg5.jsonl | python -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print('cfg5 $v', round(d['ms_per_step'],4), {n: round(v['avg_us'],1) for n,v in k.items() if n!='note'})"
done
