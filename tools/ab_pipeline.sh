set -o pipefail
mkdir -p gpurun_out
ARGS="--steps 200 --warmup 20 --no-cpu-baseline"
for v in "default:" "side:--prep-stream 1 --pipeline 0" "stepwise:--pipeline 0" "side_pipe:--prep-stream 1"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 200 python bench.py $ARGS $a > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "fail $n"; tail -5 gpurun_out/ab_$n.err; exit 1; }
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    k = r.get("kernels", {})
    print("%-14s ms/step %.4f " % (f.split("ab_")[1][:-5], r["ms_per_step"]), " ".join("%s=%.1fus" % (n, v["avg_us"]) for n, v in k.items() if isinstance(v, dict)))
PY
