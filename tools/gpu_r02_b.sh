#!/bin/bash
# Round-2 second pass: every -m gpu test, then the lane-per-pair draw A/B
# (neg_check 1 = Pos(u) set probes, one lane per pair; 0 = 8-lane row scan)
# on every config.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r02b
mkdir -p $OUT
Q="--no-cpu-baseline --no-ndcg"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_all.log 2>&1
rc=$?
tail -15 $OUT/pytest_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit 1; fi
for C in cfg2 cfg3 cfg5 cfg4; do
  for N in 0 1; do
    timeout -k 10 300 python bench.py --config $C --neg-check $N --steps 100 --warmup 10 $Q > $OUT/b_${C}_nc$N.json 2> $OUT/b_${C}_nc$N.err || { echo "$C nc$N failed"; tail -20 $OUT/b_${C}_nc$N.err; exit 1; }
    python - $OUT/b_${C}_nc$N.json <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read())
k = r["kernels"]
print(sys.argv[1].split("/")[-1], "ms/step %.4f" % r["ms_per_step"], "value %.3e" % r["value"],
      {n: round(v["avg_us"], 1) for n, v in k.items() if isinstance(v, dict)})
PY
  done
done
echo ALL DONE
