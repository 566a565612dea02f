#!/bin/bash
# Quick GPU loop: selected GPU tests (PYTEST_K) then the default bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_quick.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_quick.log
if [ $rc -ne 0 ]; then echo "PYTEST rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 200 --warmup 20 --no-cpu-baseline --no-ndcg} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_quick.err; exit 1; }
cat gpurun_out/bench_quick.json
