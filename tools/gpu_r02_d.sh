#!/bin/bash
# Round-2 fourth pass: every -m gpu test (deterministic mode fixed, item bias
# through the slot path), then cfg4 / cfg2 A/B of experiment builds.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r02d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_all.log 2>&1
rc=$?
tail -8 $OUT/pytest_all.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit 1; fi
Q="--steps 100 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0"
summ() {
python - "$1" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read())
k = r["kernels"]
print(sys.argv[1].split("/")[-1], "ms/step %.4f" % r["ms_per_step"], {n: round(v["avg_us"], 1) for n, v in k.items() if isinstance(v, dict) and v["launches"] > 1})
PY
}
for C in cfg4 cfg2; do
  for lib in collaborativefilteringusingtensorflow_amd/build/libcf_engine.so collaborativefilteringusingtensorflow_amd/build/variants/*/libcf_engine.so; do
    v=$(basename $(dirname $lib)); [ "$v" = build ] && v=default
    CF_ENGINE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config $C $Q > $OUT/ab_${C}_$v.json 2> $OUT/ab_${C}_$v.err || { echo "$C $v failed"; tail -5 $OUT/ab_${C}_$v.err; exit 1; }
    summ $OUT/ab_${C}_$v.json
  done
done
echo ALL DONE
