# fixed-point deterministic pos_sort: parity + bitwise tests, cfg2 det vs fast line
set -o pipefail
mkdir -p gpurun_out/s6
timeout -k 10 600 python -u -m pytest tests/test_gpu_det_pos_sort.py tests/test_gpu_deterministic.py tests/test_gpu_pos_sort.py "tests/test_gpu_models.py::test_cfg2_bench_batch_pos_sort_matches_oracle" -x -v --timeout 240 --timeout-method thread > gpurun_out/s6/pytest.log 2>&1 || exit 1
B="--no-cpu-baseline --no-ndcg --steps 100 --warmup 20 --secondary-batch 0"
for r in 1 2; do
timeout -k 10 200 python bench.py $B > gpurun_out/s6/cfg2_$r.json 2> gpurun_out/s6/cfg2_$r.err || exit 2
timeout -k 10 200 python bench.py $B --deterministic 1 > gpurun_out/s6/cfg2_det_$r.json 2> gpurun_out/s6/cfg2_det_$r.err || exit 3
done
