#!/bin/bash
# A quick GPU check of a change: the selected GPU tests (K), then config B's bench line.
#   K="update or B100k" bash scripts/quick_check.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/qc_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -n 30 gpurun_out/qc_pytest.log; exit 1; }
  tail -n 2 gpurun_out/qc_pytest.log
fi
timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-config-d > gpurun_out/qc_bench.log 2>&1 \
  || { echo "bench rc=$?"; tail -n 20 gpurun_out/qc_bench.log; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/qc_bench.log").read().strip().split("\n")[-1])
e = d["extra"]
print("value", d["value"], "ms", d["ms_per_step"])
print("split", e["step_split_ms"])
print("device", e["device_ms_per_step"])
print("host", {k: v for k, v in e["host_phases_ms"].items() if k.startswith(("update", "train", "accum"))})
PY
