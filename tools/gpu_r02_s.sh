#!/bin/bash
# pos_sort on the multi-rank item reduce: distributed + pos_sort GPU tests,
# then the one-rank sharded cfg2 line (RCCL, both exchanges) with it off / on
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/psort5
timeout -k 10 700 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_pos_sort.py -x -v --timeout 200 --timeout-method thread > gpurun_out/psort5/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/psort5/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/psort5/pytest.log | head; echo "PYTEST rc=$rc"; exit $rc; }
for x in allreduce rs_ag; do
for v in 0 1; do
  CF_BENCH_SHARDED=1 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 --item-exchange $x --pos-sort $v >> gpurun_out/psort5/sharded.jsonl 2>> gpurun_out/psort5/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/psort5/bench.err; exit 1; }
  tail -1 gpurun_out/psort5/sharded.jsonl | python -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print('sharded $x pos_sort=$v', round(d['ms_per_step'],4), {n: round(v['avg_us'],1) for n,v in k.items() if n!='note'})"
done
done
