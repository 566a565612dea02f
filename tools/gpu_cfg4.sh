set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config cfg4 --steps 100 --warmup 10 --no-cpu-baseline --no-ndcg > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err || { echo "cfg4 failed"; tail -20 gpurun_out/bench_cfg4.err; exit 1; }
cat gpurun_out/bench_cfg4.json
CF_DIST_BACKEND=gloo CF_SHARE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --config cfg4 --n-users 1000000 --n-items 100000 --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_cfg4_dist2.json 2> gpurun_out/bench_cfg4_dist2.err || { echo "dist rehearsal failed"; tail -30 gpurun_out/bench_cfg4_dist2.err; exit 1; }
cat gpurun_out/bench_cfg4_dist2.json
