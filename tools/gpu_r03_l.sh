#!/bin/bash
# Fused scoring: the sequential kernel with B operands read one MFMA group
# ahead (default) vs without (variant build nobpf) vs the software-pipelined
# kernel (fused_variant 1); top-k GPU tests; then rocprof of cfg3 / cfg5 on
# the current defaults (LDS gradient kernel, score pass in the cfg5 trace),
# and the 2-rank gloo rehearsal line (roofline.frac must be non-null, no
# one-GPU traffic).
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03l
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py "tests/test_gpu_bench_configs.py::test_fused_topk_d128_cfg5_slice" \
  -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -4 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
B=collaborativefilteringusingtensorflow_amd/build
A="--no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 20 --warmup 5"
cat > /tmp/psf.py <<'PY'
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1]); sp = d.get('score_pass') or {}
print(sys.argv[1], round(d['ms_per_step'], 4), 'score s', sp.get('seconds'), 'TF', sp.get('TFLOPs'), 'kernel TF', sp.get('kernel_TFLOPs'))
PY
run() {  # tag config lib extra-args...
  local tag=$1 c=$2 lib=$3; shift 3
  CF_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --config $c $A "$@" > $OUT/${c}_$tag.json 2>> $OUT/bench.err || { echo "BENCH FAILED $c $tag"; tail -20 $OUT/bench.err; exit 1; }
  python /tmp/psf.py "$c $tag" < $OUT/${c}_$tag.json | tee -a $OUT/ab.txt
}
L=$PWD/$B/libcf_engine.so
for r in 1 2; do
  run bpf$r cfg5 $L
  run nobpf$r cfg5 $PWD/$B/variants/nobpf/libcf_engine.so
  run pipe$r cfg5 $L --fused-variant 1
done
run bpf_d64 cfg2 $L --score-pass
run nobpf_d64 cfg2 $PWD/$B/variants/nobpf/libcf_engine.so --score-pass
for c in cfg3 cfg5 cfg2; do
  bash tools/gpu_profile_cfg.sh r03_$c --config $c || exit 1
done
CF_DIST_BACKEND=gloo CF_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 \
  --no-cpu-baseline --no-ndcg --secondary-batch 0 > $OUT/dist2_gloo.json 2> $OUT/dist2_gloo.err || { echo "gloo rehearsal failed"; tail -20 $OUT/dist2_gloo.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/dist2_gloo.json').read().strip().splitlines()[-1]); r=d['roofline']; print('dist2', d['n_gpus'], d['value'], 'frac', r['frac'], 'traffic', r['traffic'], r['pmc_key'])"
