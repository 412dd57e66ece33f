#!/bin/bash
# Round-5 closing measurement set (after the update-loop fixed point, the select pass and the
# pinned result downloads): the default bench line (with the reference's CPU baseline), the
# config-D line, scripts/configs.py on D1M / E9100 / C20k / C100k, then config B under
# rocprofv3 --kernel-trace --stats and the FETCH_SIZE / WRITE_SIZE passes (separate runs; the
# accumulation takes a plain launch under the profiler, MC_ACCUM_PLAIN_LAUNCH, so the profiled
# processes exit cleanly).  Every step under its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date +%s >> gpurun_out/tick.txt; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
step() { echo "$1 rc=$2 t=$(date +%s)" | tee -a gpurun_out/fin_status.txt; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python bench.py > gpurun_out/fin_bench_b.log 2>&1; step bench_b $?
timeout -k 10 600 python bench.py --workload D --steps 3 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/fin_bench_d.log 2>&1; step bench_d $?
timeout -k 10 900 python scripts/configs.py ${CFGS:-D1M E9100 C20k C100k} > gpurun_out/fin_configs.log 2>&1; step configs $?
export MC_ACCUM_PLAIN_LAUNCH=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_stats -o run -- \
  python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config-d > gpurun_out/fin_stats.log 2>&1; step stats $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/fin_fetch -o run -- \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-config-d > gpurun_out/fin_fetch.log 2>&1; step fetch $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/fin_write -o run -- \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-config-d > gpurun_out/fin_write.log 2>&1; step write $?
grep -h "^{" gpurun_out/fin_bench_b.log | tail -1 | head -c 1200; echo
