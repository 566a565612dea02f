#!/bin/bash
# GBPR on the LDS-staged kernel by default, split exchange step only at N > 1:
# the whole -m gpu suite, smoke, the cfg4 line and the one-rank sharded cfg4
# lines (serial step at one rank).
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03n
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -8 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
A="--no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 100 --warmup 10"
timeout -k 10 300 python bench.py --config cfg4 $A > $OUT/cfg4.json 2>> $OUT/bench.err || { echo "cfg4 failed"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/cfg4.json').read().strip().splitlines()[-1]); print('cfg4', d['value'], d['ms_per_step'], d['roofline']['frac'], {n: round(v['avg_us'],1) for n, v in d['kernels'].items() if isinstance(v, dict)})"
for ex in allreduce rs_ag; do
  CF_BENCH_SHARDED=1 timeout -k 10 400 python bench.py --config cfg4 $A --item-exchange $ex > $OUT/cfg4_sharded1_$ex.json 2> $OUT/cfg4_sharded1_$ex.err || { echo "cfg4 sharded $ex failed"; tail -20 $OUT/cfg4_sharded1_$ex.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/cfg4_sharded1_$ex.json').read().strip().splitlines()[-1]); print('cfg4 sharded1 $ex', d['value'], d['ms_per_step'], d['roofline']['frac'], {n: round(v['avg_us'],1) for n, v in d['kernels'].items() if isinstance(v, dict)})"
done
