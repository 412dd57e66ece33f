#!/bin/bash
# A/B of NW launch-form knobs on the training sampler (config B bench, no CPU baseline): for
# each variant (comma-separated env assignments, "base" = none) one bench run; prints the
# training phases.   VARIANTS="base MC_NW_MW_MAX=1" bash scripts/nw_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  envs=(); [ "$v" != base ] && envs=(${v//,/ })
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-config-d \
    > gpurun_out/nwab_$v.log 2>&1 || { echo "bench rc=$?"; tail -n 20 gpurun_out/nwab_$v.log; exit 1; }
  python - "$v" gpurun_out/nwab_$v.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
h = d["extra"]["host_phases_ms"]
print("%-40s ms/step %.2f train %.2f search %.2f (align %.2f) labels %.2f nw_dev %.2f clusters %d"
      % (sys.argv[1], d["ms_per_step"], h["train"], h["train.nw_search"], h["train.nw_search.align"],
         h["train.nw_labels"], d["extra"]["device_ms_per_step"]["nw"], d["extra"]["clusters"]))
PY
done
