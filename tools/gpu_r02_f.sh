#!/bin/bash
# Round-2 validation + evidence pass: smoke, every -m gpu test, the default
# bench line, rocprofv3 passes for cfg2 / cfg4, sharded one-rank lines, a
# 4-rank gloo rehearsal of the self-launched multi-GPU path.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/r02f
mkdir -p $OUT
Q="--no-cpu-baseline --no-ndcg"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_all.log 2>&1
rc=$?
tail -4 $OUT/pytest_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit 1; fi
timeout -k 10 400 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo bench failed; tail -20 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
A="--steps 60 --warmup 10 $Q --secondary-batch 0"
for C in cfg2 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${C}_trace -o run -- python bench.py --config $C $A > $OUT/${C}_trace.log 2>&1 || { echo "$C trace failed"; tail -20 $OUT/${C}_trace.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${C}_fetch -o run -- python bench.py --config $C $A --no-profile > $OUT/${C}_fetch.log 2>&1 || { echo "$C fetch failed"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${C}_write -o run -- python bench.py --config $C $A --no-profile > $OUT/${C}_write.log 2>&1 || { echo "$C write failed"; exit 1; }
  echo "$C profiled"
done
for C in cfg3 cfg5; do
  timeout -k 10 400 python bench.py --config $C --steps 100 --warmup 10 $Q > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { echo "$C failed"; tail -5 $OUT/bench_$C.err; exit 1; }
done
timeout -k 10 400 python bench.py --config cfg4 --steps 100 --warmup 10 $Q > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err || { echo "cfg4 failed"; exit 1; }
timeout -k 10 400 python bench.py --config cfg4 --batch 1048576 --steps 20 --warmup 5 $Q --secondary-batch 0 > $OUT/bench_cfg4_b1m.json 2> $OUT/bench_cfg4_b1m.err || { echo "cfg4 b1m failed"; tail -5 $OUT/bench_cfg4_b1m.err; exit 1; }
for X in allreduce rs_ag; do
  CF_BENCH_SHARDED=1 timeout -k 10 400 python bench.py --config cfg4 --item-exchange $X --steps 50 --warmup 10 $Q > $OUT/bench_cfg4_sharded1_$X.json 2> $OUT/bench_cfg4_sharded1_$X.err || { echo "cfg4 sharded $X failed"; tail -20 $OUT/bench_cfg4_sharded1_$X.err; exit 1; }
  CF_BENCH_SHARDED=1 timeout -k 10 400 python bench.py --item-exchange $X --steps 100 --warmup 10 $Q > $OUT/bench_cfg2_sharded1_$X.json 2> $OUT/bench_cfg2_sharded1_$X.err || { echo "cfg2 sharded $X failed"; tail -20 $OUT/bench_cfg2_sharded1_$X.err; exit 1; }
done
CF_DIST_BACKEND=gloo CF_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 4 --steps 10 --warmup 2 $Q --secondary-batch 0 > $OUT/bench_cfg2_dist4_gloo.json 2> $OUT/bench_cfg2_dist4_gloo.err || { echo dist4 failed; tail -20 $OUT/bench_cfg2_dist4_gloo.err; exit 1; }
python - $OUT <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    k = r.get("kernels", {})
    print(os.path.basename(f), "n=%d ms/step %.4f value %.3e" % (r["n_gpus"], r["ms_per_step"], r["value"]),
          r["config"].get("item_exchange", ""), {n: round(v["avg_us"], 1) for n, v in k.items() if isinstance(v, dict) and v["launches"] > 1})
PY
echo ALL DONE
