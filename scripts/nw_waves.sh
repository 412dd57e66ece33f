#!/bin/bash
# NW latency form at 4 / 8 / 16 waves per pair: parity (NW + e2e GPU tests) and config B / E timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in 8 16 4; do
  MC_NW_WAVES=$W timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 200 -k "nw or e2e" > gpurun_out/nw_w$W.log 2>&1 || exit $?
  MC_NW_WAVES=$W timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config-d --stats-out gpurun_out/bench_w$W.json > gpurun_out/bench_w$W.log 2>&1 || exit $?
  MC_NW_WAVES=$W timeout -k 10 300 python scripts/configs.py E91 E9100 > gpurun_out/configs_w$W.log 2>&1 || exit $?
  echo "W=$W done $(date +%s)"
done
