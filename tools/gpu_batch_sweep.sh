#!/bin/bash
# Per-GPU batch sweep of the cfg2 line: the single-GPU path and the sharded
# code path on one rank (CF_BENCH_SHARDED=1, the local cost of a multi-GPU
# step).  One JSON line per run in gpurun_out/sweep/.
set -o pipefail
mkdir -p gpurun_out/sweep
export PYTHONUNBUFFERED=1
CFG=${CFG:-cfg2}
for B in ${BATCHES:-65536 131072 262144 524288}; do
  [ -n "$SKIP_SINGLE" ] || timeout -k 10 240 python bench.py --config $CFG --batch $B --steps 100 --warmup 10 --no-cpu-baseline --no-ndcg \
    > gpurun_out/sweep/${CFG}_b${B}.json 2> gpurun_out/sweep/${CFG}_b${B}.err || { echo "FAIL $B"; tail -5 gpurun_out/sweep/${CFG}_b${B}.err; exit 1; }
  [ -n "$SKIP_SINGLE" ] || echo "single B=$B $(python -c "import json;d=json.load(open('gpurun_out/sweep/${CFG}_b${B}.json'));print(round(d['ms_per_step']*1e3,1),'us',round(d['value']/1e6),'M/s')")"
  for IR in ${ITEM_REDUCE:-1}; do
  CF_BENCH_SHARDED=1 timeout -k 10 240 python bench.py --config $CFG --batch $B --item-reduce $IR --steps 100 --warmup 10 --no-cpu-baseline --no-ndcg \
    > gpurun_out/sweep/${CFG}_b${B}_sharded_ir${IR}.json 2> gpurun_out/sweep/${CFG}_b${B}_sharded_ir${IR}.err || { echo "FAIL sharded $B"; tail -5 gpurun_out/sweep/${CFG}_b${B}_sharded_ir${IR}.err; exit 1; }
  echo "sharded B=$B item_reduce=$IR $(python -c "import json;d=json.load(open('gpurun_out/sweep/${CFG}_b${B}_sharded_ir${IR}.json'));print(round(d['ms_per_step']*1e3,1),'us',round(d['value']/1e6),'M/s', {k:round(v['avg_us'],1) for k,v in d['kernels'].items() if isinstance(v,dict)})")"
  done
done
