#!/bin/bash
# NW + e2e GPU parity, config B bench and config E runs with the default launch choices.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 200 -k "nw or e2e" > gpurun_out/nw.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config-d --stats-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 python scripts/configs.py E91 E9100 C20k > gpurun_out/configs.log 2>&1 || exit $?
