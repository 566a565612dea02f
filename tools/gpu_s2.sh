set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests/test_gpu_det_pos_sort.py tests/test_gpu_pos_sort.py tests/test_gpu_deterministic.py tests/test_gpu_models.py -x -v --timeout 240 --timeout-method thread > gpurun_out/s2/pytest.log 2>&1 || exit 1
B="--no-cpu-baseline --no-ndcg --steps 100 --warmup 20 --secondary-batch 0"
timeout -k 10 200 python bench.py $B > gpurun_out/s2/cfg2.json 2> gpurun_out/s2/cfg2.err || exit 2
timeout -k 10 200 python bench.py $B --deterministic 1 > gpurun_out/s2/cfg2_det.json 2> gpurun_out/s2/cfg2_det.err || exit 3
timeout -k 10 200 python bench.py $B --deterministic 1 --pos-sort 0 > gpurun_out/s2/cfg2_det_ps0.json 2> gpurun_out/s2/cfg2_det_ps0.err || exit 4
