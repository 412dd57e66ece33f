#!/bin/bash
# Round-4 A/B on the GPU box: config B bench lines (3 steps) per variant (an environment
# assignment; "base" = none), accumulation phase profile per variant.
#   VARIANTS="base MC_ACCUM_POLL_SLEEP=0 MC_NW_WAVES=2" bash scripts/r04_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
( while sleep 45; do date +%s >> gpurun_out/tick.txt; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
for v in ${VARIANTS:-base}; do
  envs=(); [ "$v" != base ] && envs=(${v//,/ })
  echo "== $v"
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-config-d \
    > gpurun_out/ab_$v.log 2>&1 || { echo "bench rc=$?"; tail -n 20 gpurun_out/ab_$v.log; exit 1; }
  python - gpurun_out/ab_$v.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
e = d["extra"]
print("  value %.0f ms/step %.2f roof %.4f us/step %.2f nw_ms %.2f train %.2f accum %.2f" % (
    d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["us_per_step"],
    e["nw_roofline"]["ms_per_step"], e["host_phases_ms"]["train"], e["host_phases_ms"]["accumulate"]))
PY
  if [ -n "${PROF:-}" ]; then
    env "${envs[@]}" MC_ACCUM_PROFILE=$PROF timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-d \
      > gpurun_out/ab_prof_$v.log 2>&1 || { echo "bench rc=$?"; tail -n 20 gpurun_out/ab_prof_$v.log; exit 1; }
    grep "^\[accum" gpurun_out/ab_prof_$v.log | tail -n 3
  fi
done
