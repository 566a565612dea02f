#!/bin/bash
# Same-box A/B: the previous commit's engine (variants/head) vs the working tree.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r02k
mkdir -p $OUT
Q="--steps 100 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0"
summ() {
python - "$1" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read())
k = r["kernels"]
print(sys.argv[1].split("/")[-1], "ms/step %.4f" % r["ms_per_step"], {n: round(v["avg_us"], 1) for n, v in k.items() if isinstance(v, dict) and v["launches"] > 1})
PY
}
run() { # name lib args
  local n=$1 lib=$2; shift 2
  CF_ENGINE_LIB=$PWD/$lib timeout -k 10 300 python bench.py $Q "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; tail -5 $OUT/$n.err; exit 1; }
  summ $OUT/$n.json
}
L=collaborativefilteringusingtensorflow_amd/build
for rep in 1 2; do
  run cfg2_head_$rep $L/variants/head/libcf_engine.so --config cfg2
  run cfg2_new_$rep $L/libcf_engine.so --config cfg2
done
run cfg3_head $L/variants/head/libcf_engine.so --config cfg3
run cfg3_new $L/libcf_engine.so --config cfg3
run cfg4_head $L/variants/head/libcf_engine.so --config cfg4
run cfg4_new $L/libcf_engine.so --config cfg4
run cfg2_det $L/libcf_engine.so --config cfg2 --deterministic 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_deterministic.py > $OUT/pytest_det.log 2>&1 || { echo "det tests failed"; tail -30 $OUT/pytest_det.log; exit 1; }
tail -1 $OUT/pytest_det.log
echo ALL DONE
