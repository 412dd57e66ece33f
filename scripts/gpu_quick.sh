#!/bin/bash
# A focused GPU session: named pytest selection (-k EXPR in $K), then configs (names in $CONFIGS).
# Every GPU step has its own time limit; the first failing step ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${K:-}" ]; then
  timeout -k 10 900 python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 600 --timeout-method thread \
    -p no:cacheprovider -k "$K" > gpurun_out/pytest_quick.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 15 gpurun_out/pytest_quick.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${CONFIGS:-}" ]; then
  timeout -k 10 900 python scripts/configs.py $CONFIGS > gpurun_out/configs.log 2>&1
  rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.log | cut -c1-1500
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
