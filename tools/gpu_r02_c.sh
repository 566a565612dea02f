#!/bin/bash
# Round-2 third pass: the new / changed GPU tests, then rocprofv3 evidence
# for every bench config (kernel trace + stats; FETCH_SIZE and WRITE_SIZE in
# passes of their own) and the cfg5 scoring pass kernel trace.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r02c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_configs.py tests/test_gpu_deterministic.py tests/test_gpu_sampler.py tests/test_gpu_distributed.py -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -12 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit 1; fi
A="--steps 60 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0"
for C in cfg2 cfg3 cfg4 cfg5; do
  X=""
  [ $C = cfg5 ] && X="--score-pass"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${C}_trace -o run -- python bench.py --config $C $A $X > $OUT/${C}_trace.log 2>&1 || { echo "$C trace failed"; tail -20 $OUT/${C}_trace.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${C}_fetch -o run -- python bench.py --config $C $A --no-profile > $OUT/${C}_fetch.log 2>&1 || { echo "$C fetch failed"; tail -20 $OUT/${C}_fetch.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${C}_write -o run -- python bench.py --config $C $A --no-profile > $OUT/${C}_write.log 2>&1 || { echo "$C write failed"; tail -20 $OUT/${C}_write.log; exit 1; }
  echo "$C profiled"
done
echo ALL DONE
