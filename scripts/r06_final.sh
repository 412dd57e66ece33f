#!/bin/bash
# Round-6 closing measurement set: the default bench line (the driver's command: reference CPU
# baseline at x86-64-v4 and x86-64-v3, config D beside config B), scripts/configs.py, then the
# bench under rocprofv3 --kernel-trace --stats (config B and the config-D leg: their
# accumulation kernels are different instantiations, dense and dense-streaming) and the
# FETCH_SIZE / WRITE_SIZE passes of config B (separate runs; the accumulation takes a plain
# launch under the profiler, MC_ACCUM_PLAIN_LAUNCH, so the profiled processes exit cleanly).
# Every step under its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date +%s >> gpurun_out/tick.txt; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
step() { echo "$1 rc=$2 t=$(date +%s)" | tee -a gpurun_out/fin6_status.txt; [ "$2" -eq 0 ] || exit "$2"; }
for s in ${STEPS:-bench configs stats fetch write}; do
  case $s in
    bench) timeout -k 10 900 python bench.py --stats-out gpurun_out/fin6_bench.json > gpurun_out/fin6_bench.log 2>&1; step bench $? ;;
    configs) timeout -k 10 900 python scripts/configs.py ${CFGS:-D1M E9100 E91 C20k C100k} > gpurun_out/fin6_configs.log 2>&1; step configs $? ;;
    stats) MC_ACCUM_PLAIN_LAUNCH=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin6_stats -o run -- \
             python bench.py --steps 10 --warmup 2 --no-cpu-baseline --stats-out gpurun_out/fin6_stats_bench.json > gpurun_out/fin6_stats.log 2>&1; step stats $? ;;
    fetch) MC_ACCUM_PLAIN_LAUNCH=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/fin6_fetch -o run -- \
             python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-config-d > gpurun_out/fin6_fetch.log 2>&1; step fetch $? ;;
    write) MC_ACCUM_PLAIN_LAUNCH=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/fin6_write -o run -- \
             python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-config-d > gpurun_out/fin6_write.log 2>&1; step write $? ;;
  esac
done
grep -h "^{" gpurun_out/fin6_bench.log 2>/dev/null | tail -1 | head -c 1500; echo
