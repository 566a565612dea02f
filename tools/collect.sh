#!/bin/bash
# Copy a gpu_run.sh call's outputs into profiles/<round>/<name>/ and key its
# PMC passes into profiles/pmc_traffic.json (tools/pmc_summary.py writes
# profiles/<round>/<key>_pmc_{fetch,write}.csv beside the kernel stats).
#   bash tools/collect.sh <round> <OUT of the call> <name> [prof tags...]
#   e.g. bash tools/collect.sh r04 gpurun_out/r04a final cfg2 cfg3
set -e
R=$1; G=$2; N=$3; shift 3
O=profiles/$R/$N
mkdir -p $O
for f in pytest.log smoke.log; do [ -f $G/$f ] && cp $G/$f $O/; done
for f in $G/bench_*.json; do [ -f $f ] && tail -n 1 $f > $O/$(basename $f); done
for c in "$@"; do
  P=gpurun_out/prof_$c
  [ -d $P ] || { echo "no $P"; continue; }
  tail -n 1 $P/bench.json > /tmp/collect_$c.json
  key=$(python -c "import json; print(json.load(open('/tmp/collect_$c.json'))['roofline']['pmc_key'])")
  cp /tmp/collect_$c.json profiles/$R/${key}_bench.json
  CF_ROUND=$R python tools/pmc_summary.py $key $P/fetch $P/write $P/trace > /dev/null
  st=$(find $P/trace -name "*kernel_stats.csv" | head -1); [ -n "$st" ] && cp $st profiles/$R/${key}_kernel_stats.csv
  echo "$c -> $key"
done
