#!/bin/bash
# NW iteration: NW parity tests, then config B device time per kernel family (2 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "nw or e2e" --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/nw_parity.log 2>&1 || { tail -n 30 gpurun_out/nw_parity.log; exit 1; }
tail -n 2 gpurun_out/nw_parity.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/nw_bench.log 2>&1 || { tail -n 20 gpurun_out/nw_bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads([x for x in open("gpurun_out/nw_bench.log") if x.startswith("{")][-1])
e = d["extra"]
print("value", d["value"], "ms/step", d["ms_per_step"], "nw ms", e["device_ms_per_step"]["nw"], "nw_search", e["host_phases_ms"]["train.nw_search"], "align", e["host_phases_ms"]["train.nw_search.align"], "accum us/step", d["roofline"]["us_per_step"])
PY
