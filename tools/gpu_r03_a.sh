#!/bin/bash
# r03 first GPU pass: the whole -m gpu suite with the elementwise tolerance
# (not -x: every failure is listed), the new full-size cfg2 bench-batch
# pos_sort oracle test, the exchange batch-size test, smoke, one bench line.
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
tail -30 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['pmc_key'], d['kernels'].get('step'), d['kernels'].get('apply_prep'), d['kernels'].get('psort'))"
exit $rc
