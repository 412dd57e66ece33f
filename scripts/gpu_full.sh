#!/bin/bash
# Full GPU check: the whole -m gpu suite, then the bench under rocprofv3 (kernel stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py \
  --steps 2 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/prof.log 2>&1
echo "prof rc=$?"; grep '^{' gpurun_out/prof.log | tail -c 600
