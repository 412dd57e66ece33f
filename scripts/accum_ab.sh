#!/bin/bash
# A/B of accumulation-kernel variants on the GPU box: parity first, then for each variant
# (an environment assignment, "base" = none) one plain bench run and one MC_ACCUM_PROFILE=1 run.
#   VARIANTS="base MC_ACCUM_NO_PREFETCH=1" bash scripts/accum_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "${SKIP_PARITY:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edges.py -m gpu -x -q \
    -k "e2e or device_accumulate or B100k or member_cache or update_iteration" --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/accum_parity.log 2>&1 || { echo "parity rc=$?"; tail -n 30 gpurun_out/accum_parity.log; exit 1; }
  tail -n 1 gpurun_out/accum_parity.log
fi
summ() {
  python - "$1" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print("  value %.0f ms/step %.2f roof %.4f us/step %.2f resident %.0f nw_ms %.2f"
      % (d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["us_per_step"],
         d["extra"]["resident_sequences_per_s"], d["extra"]["nw_roofline"]["ms_per_step"]))
PY
}
for v in ${VARIANTS:-base}; do
  envs=(); [ "$v" != base ] && envs=(${v//,/ })
  echo "== $v"
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-config-d \
    > gpurun_out/ab_$v.log 2>&1 || { echo "bench rc=$?"; tail -n 20 gpurun_out/ab_$v.log; exit 1; }
  summ gpurun_out/ab_$v.log
  env "${envs[@]}" MC_ACCUM_PROFILE=${PROFV:-1} timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config-d \
    > gpurun_out/ab_prof_$v.log 2>&1 || { echo "bench rc=$?"; tail -n 20 gpurun_out/ab_prof_$v.log; exit 1; }
  grep "^\[accum" gpurun_out/ab_prof_$v.log | tail -n 3 | head -n 2
done
