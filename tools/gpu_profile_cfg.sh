#!/bin/bash
# rocprofv3 kernel trace + stats and the FETCH_SIZE / WRITE_SIZE passes (one
# counter group per pass, MI355X_MICROARCH.md) of one bench configuration,
# plus the bench line itself (its roofline.pmc_key names the counters'
# entry in profiles/pmc_traffic.json: tools/pmc_summary.py <key> ...).
#   bash tools/gpu_profile_cfg.sh <tag> [bench args...]
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/prof_$TAG
mkdir -p $OUT
A="--steps 100 --warmup 10 --no-cpu-baseline --no-ndcg --secondary-batch 0 $*"
timeout -k 10 400 python bench.py $A > $OUT/bench.json 2> $OUT/bench.err || { echo "$TAG bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('$TAG', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['pmc_key'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py $A > $OUT/trace.log 2>&1 || { echo "$TAG trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python bench.py $A --no-profile > $OUT/fetch.log 2>&1 || { echo "$TAG fetch pass failed"; tail -20 $OUT/fetch.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python bench.py $A --no-profile > $OUT/write.log 2>&1 || { echo "$TAG write pass failed"; tail -20 $OUT/write.log; exit 1; }
echo "$TAG profile passes done"
