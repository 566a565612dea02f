#!/bin/bash
# Round-3 final pass (session 3) on the committed build: the whole -m gpu suite, smoke,
# the default bench line (cfg2 with the CPU baseline and the cfg1 NDCG check),
# then the rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes and the
# bench line of cfg2..cfg5 (tools/gpu_profile_cfg.sh; their pmc keys carry
# this build's digest), and the 2-rank gloo rehearsal of the sharded line.
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03final2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -8 $OUT/pytest.log
# a failing test is read afterwards; a GPU fault / abort / timeout stops here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 500 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "default bench failed"; tail -20 $OUT/bench_default.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['pmc_key'], d.get('cpu_baseline'), d.get('ndcg10_vs_ref'))"
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0 --deterministic 1 > $OUT/cfg2_det.json 2> $OUT/cfg2_det.err || { echo "det bench failed"; tail -20 $OUT/cfg2_det.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/cfg2_det.json').read().strip().splitlines()[-1]); print('det', d['value'], d['ms_per_step'])"
