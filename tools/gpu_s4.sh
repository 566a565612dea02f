# same-box A/B: main build (pair-prefetch code present, option off) vs the
# variant with the prefetch compiled out (CF_PAIR_PREFETCH=0)
set -o pipefail
mkdir -p gpurun_out/s4
B="--no-cpu-baseline --no-ndcg --steps 100 --warmup 20 --secondary-batch 0"
V=collaborativefilteringusingtensorflow_amd/build/variants/nopf/libcf_engine.so
for r in 1 2 3; do
timeout -k 10 200 python bench.py $B > gpurun_out/s4/main_$r.json 2> gpurun_out/s4/main_$r.err || exit 2
CF_ENGINE_LIB=$V timeout -k 10 200 python bench.py $B > gpurun_out/s4/nopf_$r.json 2> gpurun_out/s4/nopf_$r.err || exit 3
done
