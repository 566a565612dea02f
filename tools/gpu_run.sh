#!/bin/bash
# The GPU runner (run through gpurun).  Steps run in the order STEPS lists them
# (space separated), each under its own time limit.  A GPU fault, an abort, a
# timeout or a failed step ends the call; failing tests (pytest rc 1) do not,
# their log is read afterwards.
#
#   tests  python -m pytest $PYTEST_ARGS (default: tests -m gpu)   -> $OUT/pytest.log
#   smoke  __graft_entry__.smoke()                                  -> $OUT/smoke.log
#   bench  one bench.py line per "name:args" in $BENCH (';' list)   -> $OUT/bench_<name>.json
#          (default: "default:" = the driver's own line)
#   prof   rocprofv3 kernel trace + stats, FETCH_SIZE and WRITE_SIZE passes of
#          one bench configuration per "tag:args" in $PROF (';' list)
#          -> gpurun_out/prof_<tag>/ (tools/gpu_profile_cfg.sh)
#   pmc    one rocprofv3 --pmc pass per "name:counters" in $PMC_SETS (';' list,
#          counters space-separated, each pass within the per-block limits:
#          8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD) over bench.py $PMC_ARGS
#          -> $OUT/pmc_<name>/ (tools/pmc_summary.py or read the CSV)
#   ab     the default build against build/variants/*/ with every "name:args"
#          of $VARIANT_OPTS (';' list)                              -> $OUT/ab_<variant>_<name>.json
#
# e.g. gpurun -- 'OUT=gpurun_out/r04a STEPS="tests bench" PYTEST_ARGS="tests/test_gpu_pos_sort.py -m gpu" bash tools/gpu_run.sh'
# Logs that change a test's tolerance are copied to profiles/<round>/ with a
# DESIGN note (tools/README.md).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=${OUT:-gpurun_out/run}
mkdir -p $OUT
STEPS=${STEPS:-"tests smoke bench"}

die() { echo "$1"; exit ${2:-1}; }

step_tests() {
  timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest ${PYTEST_ARGS:-tests -m gpu} -q -rf \
      --timeout ${TEST_TIMEOUT:-150} --timeout-method thread > $OUT/pytest.log 2>&1
  local rc=$?
  tail -12 $OUT/pytest.log
  # 0 passed, 1 some tests failed: go on; anything else (abort, timeout, fault) stops here
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || die "pytest rc $rc: stopping" $rc
  TESTS_RC=$rc
}

step_smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
      || { tail -20 $OUT/smoke.log; die "smoke failed"; }
  tail -2 $OUT/smoke.log
}

step_bench() {
  local spec name args
  IFS=';' read -ra SPECS <<< "${BENCH:-default:}"
  for spec in "${SPECS[@]}"; do
    name=${spec%%:*}; args=${spec#*:}
    timeout -k 10 ${BENCH_LIMIT:-500} python bench.py $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err \
        || { tail -20 $OUT/bench_$name.err; die "bench $name failed"; }
    python - "$OUT/bench_$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
k = d.get("kernels", {})
print("%-14s %.4g %s  %.4f ms/step  frac %s  %s" % (sys.argv[2], d["value"], d["unit"], d["ms_per_step"], r.get("frac"),
      " ".join("%s=%.1fus" % (n, v["avg_us"]) for n, v in k.items() if isinstance(v, dict) and v.get("launches", 0) > 1)))
PY
  done
}

step_prof() {
  local spec tag args
  IFS=';' read -ra SPECS <<< "${PROF:-cfg2:}"
  for spec in "${SPECS[@]}"; do
    tag=${spec%%:*}; args=${spec#*:}
    bash tools/gpu_profile_cfg.sh $tag $args || die "profile $tag failed"
  done
}

step_pmc() {
  local spec name ctrs
  local ARGS=${PMC_ARGS:---steps 30 --warmup 5 --no-cpu-baseline --no-ndcg --secondary-batch 0 --no-profile}
  IFS=';' read -ra SPECS <<< "${PMC_SETS}"
  for spec in "${SPECS[@]}"; do
    name=${spec%%:*}; ctrs=${spec#*:}
    timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/pmc_$name -o run -- python bench.py $ARGS \
        > $OUT/pmc_$name.log 2>&1 || { tail -20 $OUT/pmc_$name.log; die "pmc pass $name failed"; }
    echo "pmc $name done"
  done
}

step_ab() {
  local lib v o on oa
  local ARGS=${AB_ARGS:---steps 200 --warmup 20 --no-cpu-baseline --no-ndcg --secondary-batch 0}
  IFS=';' read -ra OS <<< "${VARIANT_OPTS:-base:}"
  for lib in collaborativefilteringusingtensorflow_amd/build/libcf_engine.so \
             collaborativefilteringusingtensorflow_amd/build/variants/*/libcf_engine.so; do
    [ -f "$lib" ] || continue
    v=$(basename $(dirname $lib)); [ "$v" = build ] && v=default
    for o in "${OS[@]}"; do
      on=${o%%:*}; oa=${o#*:}
      CF_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python bench.py $ARGS $oa > $OUT/ab_${v}_$on.json 2> $OUT/ab_${v}_$on.err \
          || { tail -5 $OUT/ab_${v}_$on.err; die "variant ${v}_$on failed"; }
    done
  done
  python - "$OUT" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/ab_*.json")):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    k = r.get("kernels", {})
    print("%-26s ms/step %.4f " % (f.split("/ab_")[1][:-5], r["ms_per_step"]),
          " ".join("%s=%.1fus" % (n, v["avg_us"]) for n, v in k.items() if isinstance(v, dict) and v.get("launches", 0) > 1))
PY
}

TESTS_RC=0
for s in $STEPS; do
  case $s in
    tests) step_tests ;;
    smoke) step_smoke ;;
    bench) step_bench ;;
    prof) step_prof ;;
    pmc) step_pmc ;;
    ab) step_ab ;;
    *) die "unknown step $s" ;;
  esac
done
exit $TESTS_RC
