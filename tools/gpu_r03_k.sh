#!/bin/bash
# LDS-staged d=128 gradient kernel and the software-pipelined fused scoring
# kernel: their GPU tests, then same-box A/B of cfg5 / cfg3 over grad_path 0
# (LDS kernel) / 2 (phased) / 1 (generic) and the 3- / 4-waves-per-SIMD
# builds, and cfg5's score pass with fused_variant 0 (pipelined) / 1.
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lds_grad.py tests/test_gpu_topk.py tests/test_gpu_bench_configs.py \
  tests/test_gpu_ensemble.py -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -8 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
B=collaborativefilteringusingtensorflow_amd/build
A="--no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 100 --warmup 10"
cat > /tmp/psf.py <<'PY'
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1]); k = d['kernels']
sp = d.get('score_pass') or {}
print(sys.argv[1], round(d['ms_per_step'], 4), {n: round(v['avg_us'], 1) for n, v in k.items() if isinstance(v, dict)},
      'score_TF', sp.get('TFLOPs'), sp.get('kernel_TFLOPs'))
PY
run() {  # tag config lib extra-args...
  local tag=$1 c=$2 lib=$3; shift 3
  CF_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --config $c $A "$@" > $OUT/${c}_$tag.json 2>> $OUT/bench.err || { echo "BENCH FAILED $c $tag"; tail -20 $OUT/bench.err; exit 1; }
  python /tmp/psf.py "$c $tag" < $OUT/${c}_$tag.json | tee -a $OUT/ab.txt
}
L=$PWD/$B/libcf_engine.so
run gp0 cfg5 $L --grad-path 0
run gp2 cfg5 $L --grad-path 2
run fv1 cfg5 $L --grad-path 0 --fused-variant 1
run lw3 cfg5 $PWD/$B/variants/lw3/libcf_engine.so --grad-path 0
run lw4 cfg5 $PWD/$B/variants/lw4/libcf_engine.so --grad-path 0
run gp0 cfg3 $L --grad-path 0
run gp1 cfg3 $L --grad-path 1
run lw3 cfg3 $PWD/$B/variants/lw3/libcf_engine.so --grad-path 0
run lw4 cfg3 $PWD/$B/variants/lw4/libcf_engine.so --grad-path 0
run gp0b cfg5 $L --grad-path 0
run gp2b cfg5 $L --grad-path 2
