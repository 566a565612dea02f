#!/bin/bash
# r03 (session 2) first GPU pass on the rebuilt tree: the whole -m gpu suite
# (not -x: every failure listed), smoke, then the rocprofv3 kernel trace +
# FETCH_SIZE / WRITE_SIZE passes and bench line of cfg2..cfg5 with the defaults
# that now run (tools/gpu_profile_cfg.sh).
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for c in cfg2 cfg3 cfg4 cfg5; do
  bash tools/gpu_profile_cfg.sh r03_$c --config $c || exit 1
done
