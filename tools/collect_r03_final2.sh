#!/bin/bash
# copy the round-3 final-pass outputs (tools/gpu_r03_final2*.sh) into
# profiles/r03/ and key the PMC passes into profiles/pmc_traffic.json
# (tools/pmc_summary.py writes profiles/r03/<key>_pmc_{fetch,write}.csv)
set -e
O=profiles/r03/final2
mkdir -p $O
G=gpurun_out/r03final2
for f in pytest.log smoke.log; do [ -f $G/$f ] && cp $G/$f $O/; done
for f in bench_default cfg2_det dist2_gloo; do [ -f $G/$f.json ] && tail -n 1 $G/$f.json > $O/$f.json; done
for c in cfg2 cfg3 cfg4 cfg5; do
  P=gpurun_out/prof_r03g_$c
  [ -d $P ] || continue
  tail -n 1 $P/bench.json > /tmp/$c.json
  key=$(python -c "import json; print(json.load(open('/tmp/$c.json'))['roofline']['pmc_key'])")
  cp /tmp/$c.json profiles/r03/${key}_bench.json
  CF_ROUND=r03 python tools/pmc_summary.py $key $P/fetch $P/write $P/trace > /dev/null
  st=$(find $P/trace -name "*kernel_stats.csv" | head -1); [ -n "$st" ] && cp $st profiles/r03/${key}_kernel_stats.csv
  echo "$c -> $key"
done
