#!/bin/bash
# pos_sort default (auto): rocprof kernel trace + FETCH/WRITE passes at cfg2,
# and the batch-size A/B that sets the auto threshold
set -o pipefail
mkdir -p gpurun_out/psort
export PYTHONUNBUFFERED=1
TAG=cfg2_psort bash tools/gpu_profile.sh || exit 1
for B in 65536 16384; do
for v in 0 1; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --no-ndcg --secondary-batch 0 --batch $B --pos-sort $v >> gpurun_out/psort/batch_ab.jsonl 2>> gpurun_out/psort/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/psort/bench.err; exit 1; }
  tail -1 gpurun_out/psort/batch_ab.jsonl | python -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernels']; print('B=$B pos_sort=$v', round(d['ms_per_step'],4), {n: round(v['avg_us'],1) for n,v in k.items() if n!='note'})"
done
done
