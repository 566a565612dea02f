#!/bin/bash
# Split GBPR exchange step (cf_xchg_grad_part / cf_xchg_finish_items): its GPU
# tests (two ranks on one device with gloo, both exchanges, split and serial)
# and the one-rank sharded cfg4 line (CF_BENCH_SHARDED=1, RCCL); the fused
# scoring kernels without B prefetch (sequential default vs pipelined) on cfg5.
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03m
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_group_exchange.py tests/test_gpu_distributed.py tests/test_gpu_topk.py tests/test_gpu_lds_grad.py \
  -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -6 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
A="--no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 50 --warmup 5"
for ex in allreduce rs_ag; do
  CF_BENCH_SHARDED=1 timeout -k 10 400 python bench.py --config cfg4 $A --item-exchange $ex > $OUT/cfg4_sharded1_$ex.json 2> $OUT/cfg4_sharded1_$ex.err || { echo "cfg4 sharded $ex failed"; tail -20 $OUT/cfg4_sharded1_$ex.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/cfg4_sharded1_$ex.json').read().strip().splitlines()[-1]); print('cfg4 sharded1 $ex', d['value'], d['ms_per_step'], d['roofline']['frac'], {n: round(v['avg_us'],1) for n, v in d['kernels'].items() if isinstance(v, dict)})"
done
for v in 0 1; do
  timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 20 --warmup 5 --fused-variant $v > $OUT/cfg5_fv$v.json 2>> $OUT/bench.err || { echo "cfg5 fv$v failed"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/cfg5_fv$v.json').read().strip().splitlines()[-1]); print('cfg5 fv$v', d['score_pass']['TFLOPs'], d['score_pass']['kernel_TFLOPs'])"
done
# cfg4 on the LDS-staged GBPR kernel (grad_path 3) vs the phased default
for gp in 0 3 0; do
  timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 100 --warmup 10 --grad-path $gp > $OUT/cfg4_gp$gp.json 2>> $OUT/bench.err || { echo "cfg4 gp$gp failed"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/cfg4_gp$gp.json').read().strip().splitlines()[-1]); print('cfg4 gp$gp', d['ms_per_step'], d['roofline']['frac'], {n: round(v['avg_us'],1) for n, v in d['kernels'].items() if isinstance(v, dict)})"
done
