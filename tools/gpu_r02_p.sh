#!/bin/bash
# pos_sort with contiguous sorted records: parity tests, then on one box the
# A/B at 2^19 / 2^18 / 2^17 pairs and FETCH/WRITE passes with the option on
# and off
set -o pipefail
mkdir -p gpurun_out/psort2
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pos_sort.py -x -q --timeout 120 --timeout-method thread > gpurun_out/psort2/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/psort2/pytest.log; [ $rc -ne 0 ] && { echo "PYTEST rc=$rc"; exit $rc; }
for B in 524288 262144 131072; do
for v in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 --batch $B --pos-sort $v >> gpurun_out/psort2/ab.jsonl 2>> gpurun_out/psort2/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/psort2/bench.err; exit 1; }
  tail -1 gpurun_out/psort2/ab.jsonl | python -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print('B=$B pos_sort=$v', round(d['ms_per_step'],4), {n: round(v['avg_us'],1) for n,v in k.items() if n!='note'})"
done
done
for v in 1 0; do
TAG=psort$v BENCH_ARGS="--steps 100 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0 --pos-sort $v" bash tools/gpu_profile.sh > /dev/null || exit 1
done
echo done
