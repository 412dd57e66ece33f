#!/bin/bash
# Round-5 full GPU check: the whole -m gpu suite (a ticker keeps gpurun_out/ fresh through the
# long config tests), then smoke().  Each step under its own limit; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date +%s >> gpurun_out/tick.txt; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -x --timeout 1300 --timeout-method thread -p no:cacheprovider \
  --durations=25 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 3 gpurun_out/smoke.log
exit $rc
