#!/bin/bash
# Extra GPU measurements: CML (cfg3) and AMF (cfg5, with the full scoring
# pass) bench lines, and a 2-rank rehearsal of the multi-GPU path on one
# device (gloo all-reduce of the bound item-gradient tensor).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py --config cfg3 --steps 100 --warmup 10 --no-cpu-baseline --no-ndcg > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err || { echo "cfg3 failed"; tail -5 gpurun_out/bench_cfg3.err; exit 1; }
cat gpurun_out/bench_cfg3.json
timeout -k 10 600 python bench.py --config cfg5 --steps 100 --warmup 10 --no-cpu-baseline --no-ndcg > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || { echo "cfg5 failed"; tail -5 gpurun_out/bench_cfg5.err; exit 1; }
cat gpurun_out/bench_cfg5.json
CF_DIST_BACKEND=gloo CF_SHARE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err || { echo "dist rehearsal failed"; tail -20 gpurun_out/bench_dist2.err; exit 1; }
cat gpurun_out/bench_dist2.json
