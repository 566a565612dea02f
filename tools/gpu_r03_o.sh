#!/bin/bash
# Dense item-row apply on the slot-row / record path (dense_apply): its GPU
# tests and the bench-config tests, then same-box A/B of cfg3 / cfg5 with
# dense_apply 1 / 0 (engine option through CF_DENSE_APPLY), then cfg4 lines.
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03o
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_lds_grad.py tests/test_gpu_bench_configs.py tests/test_gpu_step_parity.py \
  tests/test_gpu_pipeline.py -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -6 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
A="--no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 100 --warmup 10"
for r in 1 2; do
for c in cfg5 cfg3; do
  for da in 1 0; do
    CF_DENSE_APPLY=$da timeout -k 10 300 python bench.py --config $c $A > $OUT/${c}_da${da}_$r.json 2>> $OUT/bench.err || { echo "BENCH FAILED $c da$da"; tail -20 $OUT/bench.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${c}_da${da}_$r.json').read().strip().splitlines()[-1]); print('$c da$da', d['ms_per_step'], {n: round(v['avg_us'],1) for n, v in d['kernels'].items() if isinstance(v, dict)})" | tee -a $OUT/ab.txt
  done
done
done
timeout -k 10 300 python bench.py --config cfg4 $A > $OUT/cfg4.json 2>> $OUT/bench.err || { echo "cfg4 failed"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/cfg4.json').read().strip().splitlines()[-1]); print('cfg4', d['value'], d['ms_per_step'], d['roofline']['frac'], {n: round(v['avg_us'],1) for n, v in d['kernels'].items() if isinstance(v, dict)})"
for ex in allreduce rs_ag; do
  CF_BENCH_SHARDED=1 timeout -k 10 400 python bench.py --config cfg4 $A --item-exchange $ex > $OUT/cfg4_sharded1_$ex.json 2> $OUT/cfg4_sharded1_$ex.err || { echo "cfg4 sharded $ex failed"; tail -20 $OUT/cfg4_sharded1_$ex.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/cfg4_sharded1_$ex.json').read().strip().splitlines()[-1]); print('cfg4 sharded1 $ex', d['value'], d['ms_per_step'], d['roofline']['frac'], {n: round(v['avg_us'],1) for n, v in d['kernels'].items() if isinstance(v, dict)})"
done
