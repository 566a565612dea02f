#!/bin/bash
# look-back scan launch: pos_sort / distributed / step-parity tests, the cfg2
# line (psort time), and the waves-per-EU 4 variant A/B at cfg3 / cfg5
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/v
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/v/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/v/pytest.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/v/pytest.log | head; echo "PYTEST rc=$rc"; exit $rc; }
cat > /tmp/psf.py <<'PY'
import sys, json
d = json.loads(sys.stdin.read()); k = d['kernels']
print(sys.argv[1], round(d['ms_per_step'], 4), {n: round(v['avg_us'], 1) for n, v in k.items() if n != 'note'})
PY
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 >> gpurun_out/v/cfg2.jsonl 2>> gpurun_out/v/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/v/bench.err; exit 1; }
  tail -1 gpurun_out/v/cfg2.jsonl | python /tmp/psf.py cfg2
done
for c in cfg5 cfg3; do
for lib in collaborativefilteringusingtensorflow_amd/build/libcf_engine.so collaborativefilteringusingtensorflow_amd/build/variants/wpe4/libcf_engine.so; do
  CF_ENGINE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 >> gpurun_out/v/$c.jsonl 2>> gpurun_out/v/bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/v/bench.err; exit 1; }
  tail -1 gpurun_out/v/$c.jsonl | python /tmp/psf.py "$c $(basename $(dirname $lib))"
done
done
