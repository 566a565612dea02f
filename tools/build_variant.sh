#!/bin/bash
# A/B variant of libcf_engine.so that recompiles only the named sources with
# extra flags and reuses the default build's other objects:
#   bash tools/build_variant.sh <name> "<flags>" cf_eval.hip [cf_engine.cpp ...]
# -> collaborativefilteringusingtensorflow_amd/build/variants/<name>/libcf_engine.so
# (load it with CF_ENGINE_LIB; the default build must be current first).
set -e
name=$1; flags=$2; shift 2
d=collaborativefilteringusingtensorflow_amd/build
mkdir -p $d/variants/$name
rm -f $d/variants/$name/*.o $d/variants/$name/libcf_engine.so
cp -p $d/*.o $d/variants/$name/
for s in "$@"; do rm -f $d/variants/$name/$s.o; done
CF_BUILD_VARIANT=$name CF_EXTRA_FLAGS="$flags" python -m collaborativefilteringusingtensorflow_amd.csrc.build
