#!/bin/bash
# One accumulation-kernel iteration on the GPU box: parity (e2e byte-identical, device loop ==
# step loop, config B partition) then the per-step phase profile at config B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edges.py -m gpu -x -q \
  -k "e2e or device_accumulate or B100k or member_cache" --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/accum_parity.log 2>&1 || { echo "parity rc=$?"; tail -n 30 gpurun_out/accum_parity.log; exit 1; }
tail -n 3 gpurun_out/accum_parity.log
MC_ACCUM_PROFILE=${PROF:-2} timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config-d \
  > gpurun_out/accum_prof.log 2>&1 || { echo "bench rc=$?"; tail -n 30 gpurun_out/accum_prof.log; exit 1; }
grep -v '^{' gpurun_out/accum_prof.log | tail -n 4
python - <<'PY'
import json
l = [x for x in open("gpurun_out/accum_prof.log") if x.startswith("{")][-1]
d = json.loads(l)
print("value", d["value"], "ms/step", d["ms_per_step"], "roof", d["roofline"]["frac"], "us/step", d["roofline"]["us_per_step"],
      "resident", d["extra"]["resident_sequences_per_s"])
PY
