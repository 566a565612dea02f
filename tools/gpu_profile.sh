#!/bin/bash
# rocprofv3 passes over the default bench workload: kernel trace + stats, then
# one PMC pass per TCC counter (FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 100 --warmup 10 --no-cpu-baseline --no-ndcg}
TAG=${TAG:-cfg2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_trace -o run -- python bench.py $ARGS > $OUT/prof_${TAG}_trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/prof_${TAG}_trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_${TAG}_fetch -o run -- python bench.py $ARGS --no-profile > $OUT/prof_${TAG}_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/prof_${TAG}_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_${TAG}_write -o run -- python bench.py $ARGS --no-profile > $OUT/prof_${TAG}_write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/prof_${TAG}_write.log; exit 1; }
echo "profile passes done"
find $OUT/prof_${TAG}_trace -name "*stats*" | head
