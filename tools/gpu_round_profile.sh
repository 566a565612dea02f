#!/bin/bash
# Round-end measurement set: the default bench line (with the CPU baselines),
# rocprofv3 kernel trace + stats and the FETCH_SIZE / WRITE_SIZE passes of the
# same command, then the cfg3 / cfg5 bench lines.  Summaries are copied into
# profiles/ by hand afterwards (gpurun_out/ is scratch).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/rp_bench_cfg2.json 2> $OUT/rp_bench_cfg2.err || { echo "bench failed"; tail -20 $OUT/rp_bench_cfg2.err; exit 1; }
cat $OUT/rp_bench_cfg2.json
A="--steps 100 --warmup 10 --no-cpu-baseline --no-ndcg"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rp_trace -o run -- python bench.py $A > $OUT/rp_trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/rp_trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/rp_fetch -o run -- python bench.py $A --no-profile > $OUT/rp_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/rp_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/rp_write -o run -- python bench.py $A --no-profile > $OUT/rp_write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/rp_write.log; exit 1; }
echo "profile passes done"
timeout -k 10 400 python bench.py --config cfg3 $A > $OUT/rp_bench_cfg3.json 2> $OUT/rp_bench_cfg3.err || { echo "cfg3 failed"; tail -5 $OUT/rp_bench_cfg3.err; exit 1; }
timeout -k 10 600 python bench.py --config cfg5 $A > $OUT/rp_bench_cfg5.json 2> $OUT/rp_bench_cfg5.err || { echo "cfg5 failed"; tail -5 $OUT/rp_bench_cfg5.err; exit 1; }
echo "all done"
