#!/bin/bash
# Round-5 measurement set: the default bench line (with the reference's CPU baseline), the
# config-D line, and scripts/configs.py on D1M / E9100 / C20k / C100k.  Every step under its own
# limit; a ticker keeps gpurun_out/ fresh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while sleep 45; do date +%s >> gpurun_out/tick.txt; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
timeout -k 10 600 python bench.py > gpurun_out/final_bench_b.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --workload D --steps 3 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/final_bench_d.log 2>&1 || exit 1
timeout -k 10 1100 python scripts/configs.py ${CFGS:-D1M E9100 C20k C100k} > gpurun_out/final_configs.log 2>&1 || exit 1
grep -h "^{" gpurun_out/final_bench_b.log | tail -1 | head -c 1500; echo
