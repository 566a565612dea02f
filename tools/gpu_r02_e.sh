#!/bin/bash
# Round-2 A/B: cfg4 (GBPR) gradient experiments and option sets, cfg2 checks.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r02e
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
run cfg4_default $L/libcf_engine.so --config cfg4
run cfg4_biasatomic $L/libcf_engine.so --config cfg4 --bias-slots 0
run cfg4_accalways $L/variants/accalways/libcf_engine.so --config cfg4
run cfg4_p2w5 $L/variants/p2w5/libcf_engine.so --config cfg4
run cfg4_negset $L/libcf_engine.so --config cfg4 --neg-check 1
run cfg4_det $L/libcf_engine.so --config cfg4 --deterministic 1
run cfg2_default $L/libcf_engine.so --config cfg2
run cfg2_negset $L/libcf_engine.so --config cfg2 --neg-check 1
run cfg2_prepside $L/libcf_engine.so --config cfg2 --pipeline 0 --prep-stream 1
run cfg2_det $L/libcf_engine.so --config cfg2 --deterministic 1
run cfg5_default $L/libcf_engine.so --config cfg5
run cfg5_accalways $L/variants/accalways/libcf_engine.so --config cfg5
run cfg5_p2w5 $L/variants/p2w5/libcf_engine.so --config cfg5
echo ALL DONE
