# round-3 session 3: pair-record prefetch A/B + parity, deterministic pos_sort profile
set -o pipefail
mkdir -p gpurun_out/s3
timeout -k 10 600 python -u -m pytest tests/test_gpu_det_pos_sort.py tests/test_gpu_pos_sort.py tests/test_gpu_sampler.py "tests/test_gpu_models.py::test_cfg2_bench_batch_pos_sort_matches_oracle" -x -v --timeout 240 --timeout-method thread > gpurun_out/s3/pytest.log 2>&1 || exit 1
B="--no-cpu-baseline --no-ndcg --steps 100 --warmup 20 --secondary-batch 0"
for r in 1 2; do
timeout -k 10 200 python bench.py $B --pair-prefetch 1 > gpurun_out/s3/cfg2_pf1_$r.json 2> gpurun_out/s3/cfg2_pf1_$r.err || exit 2
timeout -k 10 200 python bench.py $B --pair-prefetch 0 > gpurun_out/s3/cfg2_pf0_$r.json 2> gpurun_out/s3/cfg2_pf0_$r.err || exit 3
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s3/prof_det -o det -- python bench.py $B --steps 30 --deterministic 1 > gpurun_out/s3/prof_det.log 2>&1 || exit 4
