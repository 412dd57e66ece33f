#!/bin/bash
# Kernel timeline of config B under rocprofv3 --kernel-trace (plain accumulation launch, so the
# process exits cleanly), with the parser's phase laps: where the GPU idles inside a step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp MC_ACCUM_PLAIN_LAUNCH=1 MC_PARSE_PROFILE=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_b -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/trace_b.log 2>&1
rc=$?; echo "trace rc=$rc"; grep "\[parse\]" gpurun_out/trace_b.log | tail -n 6
exit $rc
