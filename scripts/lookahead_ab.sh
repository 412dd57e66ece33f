#!/bin/bash
# Training binary search: NW decision-tree levels per dependent round (MC_NW_LOOKAHEAD), with
# the e2e parity tests first, then the bench per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q \
  -k "e2e or B100k or E91" --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/look_parity.log 2>&1 || { echo "parity rc=$?"; tail -n 30 gpurun_out/look_parity.log; exit 1; }
tail -n 1 gpurun_out/look_parity.log
for L in ${LOOKS:-1 2 3}; do
  extra=(); [[ "$L" == *,* ]] && extra=(${L#*,})   # "3,MC_NW_MW_MAX=2048": look 3 plus that setting
  env MC_NW_LOOKAHEAD=${L%%,*} "${extra[@]}" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/look_$L.log 2>&1 || exit 1
  python - gpurun_out/look_$L.log $L <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
e = d["extra"]; h = e["host_phases_ms"]
print("look", sys.argv[2], "value %.0f ms/step %.2f nw_ms %.2f nw_launches %.0f search %.2f (resolve %.2f spec %.2f align %.2f) train %.2f"
      % (d["value"], d["ms_per_step"], e["nw_roofline"]["ms_per_step"], e["launches_per_step"]["nw"],
         h["train.nw_search"], h["train.nw_search.resolve"], h["train.nw_search.speculate"], h["train.nw_search.align"], h["train"]))
PY
done
