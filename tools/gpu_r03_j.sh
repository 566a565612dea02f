#!/bin/bash
# LDS-staged d=128 gradient kernel: the whole -m gpu suite (new
# test_gpu_lds_grad.py included), smoke, then same-box A/B of cfg3 / cfg5
# over grad_path 0 (LDS kernel, compiler's registers) / 2 (phased) / 1
# (generic) and the 3- / 4-waves-per-SIMD builds; then the rocprof passes of
# cfg2 and cfg4 (not on this kernel).
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03j
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
B=collaborativefilteringusingtensorflow_amd/build
A="--no-cpu-baseline --no-ndcg --secondary-batch 0 --steps 100 --warmup 10"
cat > /tmp/psf.py <<'PY'
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1]); k = d['kernels']
print(sys.argv[1], round(d['ms_per_step'], 4), {n: round(v['avg_us'], 1) for n, v in k.items() if isinstance(v, dict)})
PY
for r in 1 2; do
for c in cfg5 cfg3; do
  for v in gp0 gp2 gp1 lw3 lw4; do
    lib=$PWD/$B/libcf_engine.so; gp=${v#gp}
    case $v in lw*) lib=$PWD/$B/variants/$v/libcf_engine.so; gp=0;; esac
    CF_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --config $c $A --grad-path $gp > $OUT/${c}_$v.json 2>> $OUT/bench.err || { echo "BENCH FAILED $c $v"; tail -20 $OUT/bench.err; exit 1; }
    python /tmp/psf.py "$c $v" < $OUT/${c}_$v.json | tee -a $OUT/ab.txt
  done
done
done
for c in cfg2 cfg4; do
  bash tools/gpu_profile_cfg.sh r03_$c --config $c || exit 1
done
