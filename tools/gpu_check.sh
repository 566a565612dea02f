#!/bin/bash
# GPU check used with gpurun: smoke -> gpu tests -> bench; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "PYTEST ABORTED rc=$rc"; exit $rc; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
exit $rc
