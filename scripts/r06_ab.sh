#!/bin/bash
# A/B of environment variants on config B (no reference baseline, no config D): for each variant
# (comma-separated assignments, "base" = none) one bench run of $STEPS steps; prints ms per step,
# the accumulation's us per step, the training's phases and the device time per family.
#   VARIANTS="base MC_NW_LOOKAHEAD=3" bash scripts/r06_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  envs=(); [ "$v" != base ] && envs=(${v//,/ })
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-config-d \
    --stats-out gpurun_out/ab6_$v.json > gpurun_out/ab6_$v.log 2>&1 || { echo "bench $v rc=$?"; tail -n 20 gpurun_out/ab6_$v.log; exit 1; }
  python - "gpurun_out/ab6_$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["line"]
e = d["extra"]
h = e["host_phases_ms"]
print("%-40s ms/step %.2f  accum us/step %.2f  train %.2f (search %.2f resolve %.2f align %.2f labels %.2f sample %.2f)  parse %.2f write %.2f"
      % (sys.argv[2], d["ms_per_step"], d["roofline"]["us_per_step"], h.get("train", 0), h.get("train.nw_search", 0),
         h.get("train.nw_search.resolve", 0), h.get("train.nw_search.align", 0), h.get("train.nw_labels", 0),
         h.get("train.sample", 0), e["step_split_ms"]["parse"], e["step_split_ms"]["write_clstr"]))
print("   device", json.dumps(e["device_ms_per_step"]), "launches", json.dumps(e["launches_per_step"]))
PY
done
