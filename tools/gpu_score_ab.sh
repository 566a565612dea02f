#!/bin/bash
# A/B of the fused scoring pass (cfg5: 1M x 100K, d=128, top-10) over the
# default build and build/variants/*; prints the score_pass line of each.
set -o pipefail
mkdir -p gpurun_out
for lib in collaborativefilteringusingtensorflow_amd/build/libcf_engine.so collaborativefilteringusingtensorflow_amd/build/variants/*/libcf_engine.so; do
  [ -f "$lib" ] || continue
  v=$(basename $(dirname $lib)); [ "$v" = build ] && v=default
  CF_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config ${CFG:-cfg5} --score-pass --steps 3 --warmup 1 --no-cpu-baseline --no-ndcg --no-profile \
    > gpurun_out/sab_$v.json 2> gpurun_out/sab_$v.err || { echo "variant $v failed"; tail -5 gpurun_out/sab_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/sab_$v.json'))['score_pass'];print(round(d['seconds'],4),'s',round(d['TFLOPs'],1),'TF/s')")"
done
