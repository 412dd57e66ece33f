#!/bin/bash
# A/B of environment variants on config D (bench.py --workload D, no reference baseline): per
# variant (comma-separated assignments, "base" = none) one run; prints ms per step, the
# accumulation kernel's ms and its HBM fraction.
#   VARIANTS="base MC_ACCUM_DRES=0" bash scripts/d_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  envs=(); [ "$v" != base ] && envs=(${v//,/ })
  env "${envs[@]}" timeout -k 10 300 python bench.py --workload D --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline \
    > gpurun_out/dab_$v.log 2>&1 || { echo "bench $v rc=$?"; tail -n 20 gpurun_out/dab_$v.log; exit 1; }
  python - "gpurun_out/dab_$v.log" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"] or {}
print("%-32s ms/step %.1f  accum launch ms %.1f  frac %.3f  clusters %s" % (sys.argv[2], d["ms_per_step"],
      r.get("avg_launch_us", 0) / 1e3, r.get("frac", 0), d["extra"].get("clusters")))
PY
done
