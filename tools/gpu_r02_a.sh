#!/bin/bash
# Round-2 first GPU pass: smoke, the new / changed GPU tests, the default
# bench line, the self-launched 2-rank line (gloo, one device), the one-rank
# RCCL sharded lines (both item exchanges), the cfg4 sharded line.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r02a
mkdir -p $OUT
Q="--no-cpu-baseline --no-ndcg"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_configs.py tests/test_gpu_distributed.py tests/test_gpu_group_exchange.py -v --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1
rc=$?
tail -25 $OUT/pytest_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit 1; fi
timeout -k 10 400 python bench.py > $OUT/b_cfg2.json 2> $OUT/b_cfg2.err || { echo bench failed; tail -20 $OUT/b_cfg2.err; exit 1; }
cat $OUT/b_cfg2.json
CF_DIST_BACKEND=gloo CF_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 $Q > $OUT/b_cfg2_dist2_gloo.json 2> $OUT/b_cfg2_dist2_gloo.err || { echo dist2 failed; tail -20 $OUT/b_cfg2_dist2_gloo.err; exit 1; }
cat $OUT/b_cfg2_dist2_gloo.json
for X in allreduce rs_ag; do
  CF_BENCH_SHARDED=1 timeout -k 10 400 python bench.py --item-exchange $X $Q > $OUT/b_cfg2_sharded1_$X.json 2> $OUT/b_cfg2_sharded1_$X.err || { echo sharded $X failed; tail -20 $OUT/b_cfg2_sharded1_$X.err; exit 1; }
  cat $OUT/b_cfg2_sharded1_$X.json
done
for X in allreduce rs_ag; do
  CF_BENCH_SHARDED=1 timeout -k 10 500 python bench.py --config cfg4 --item-exchange $X --steps 50 --warmup 10 $Q > $OUT/b_cfg4_sharded1_$X.json 2> $OUT/b_cfg4_sharded1_$X.err || { echo cfg4 sharded $X failed; tail -20 $OUT/b_cfg4_sharded1_$X.err; exit 1; }
  cat $OUT/b_cfg4_sharded1_$X.json
done
echo ALL DONE
