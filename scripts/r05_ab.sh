#!/bin/bash
# Round-5 accumulation A/B: parity of the variants under test first (config B against the
# reference's partition, e2e goldens), then scripts/r04_ab.sh's bench lines per variant.
#   K="help" VARIANTS="base MC_ACCUM_HELPERS=1" bash scripts/r05_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q \
    -k "$K" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_parity.log 2>&1 \
    || { echo "parity rc=$?"; tail -n 30 gpurun_out/ab_parity.log; exit 1; }
  tail -n 2 gpurun_out/ab_parity.log
fi
bash scripts/r04_ab.sh
