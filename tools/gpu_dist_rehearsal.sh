#!/bin/bash
# 2-rank rehearsal of the driver's N=2 bench command on ONE device (gloo,
# both ranks on device 0): the sharded step end to end, and that stdout holds
# exactly one JSON line.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
CF_DIST_BACKEND=gloo CF_SHARE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err || { echo "dist rehearsal failed"; tail -20 gpurun_out/bench_dist2.err; exit 1; }
echo "stdout lines: $(wc -l < gpurun_out/bench_dist2.json)"
python -c "import json; [json.loads(l) for l in open('gpurun_out/bench_dist2.json')]" || { echo "stdout is not JSON lines"; exit 1; }
cat gpurun_out/bench_dist2.json
