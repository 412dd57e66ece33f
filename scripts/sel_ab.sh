#!/bin/bash
# The training's selects (split.hip): the split tests, a per-call phase profile
# (MC_SPLIT_PROFILE) of one config-B step, then config B under rocprofv3 --kernel-trace --stats
# (last: rocprofv3's exit-time fault, DESIGN.md §5, ends the call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/sel_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -n 30 gpurun_out/sel_pytest.log; exit 1; }
tail -n 2 gpurun_out/sel_pytest.log
MC_SPLIT_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-d \
  > gpurun_out/sel_split_prof.log 2>&1 || { echo "split prof rc=$?"; tail -n 20 gpurun_out/sel_split_prof.log; exit 1; }
grep "\[split\]" gpurun_out/sel_split_prof.log | tail -n 12
[ -n "${ONLY_PROF:-}" ] && exit 0
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-config-d > gpurun_out/sel_bench.log 2>&1 \
  || { echo "bench rc=$?"; tail -n 20 gpurun_out/sel_bench.log; exit 1; }
tail -n 1 gpurun_out/sel_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sel_prof -o run -- \
  python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/sel_prof.log 2>&1
echo "rocprof rc=$?"
f=$(find gpurun_out/sel_prof -name "*kernel_stats.csv" | head -n 1)
[ -n "$f" ] && grep -E "select_kernel|mean_shift_kernel|Name" "$f" | cut -c1-200
exit 0
