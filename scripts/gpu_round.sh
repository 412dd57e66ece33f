#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> bench (small, then config B) -> rocprof.
# Each GPU step has its own time limit; a crash/timeout (exit > 1) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${*:-smoke pytest bench_small bench}"
status() { echo "$1 rc=$2 t=$(date +%s)" | tee -a gpurun_out/status.txt; }
# a progress tick under gpurun_out/ while long quiet steps run (input generation, D-sized benches)
( while sleep 45; do date +%s >> gpurun_out/tick.txt; done ) &
TICK=$!
trap 'kill $TICK 2>/dev/null' EXIT
for s in $STEPS; do
  case $s in
    configs) timeout -k 10 1500 python scripts/configs.py ${CONFIGS:-E91 C20k E9100 C20k_m15} > gpurun_out/configs.log 2>&1 ;;
    e2e) timeout -k 10 300 python scripts/e2e_quick.py a1k b3k30 m2k_id80 fam2k fam2k_id85 > gpurun_out/e2e.log 2>&1 ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    pytest) timeout -k 10 1500 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 900 --timeout-method thread --durations=25 > gpurun_out/pytest_gpu.log 2>&1 ;;
    pytest_k) timeout -k 10 1200 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 900 --timeout-method thread -k "${PYK}" > gpurun_out/pytest_k.log 2>&1 ;;
    bench_d_rehearsal) MC_BENCH_ONE_GPU=1 timeout -k 10 1200 python bench.py --gpus 2 --workload D --steps 2 --warmup 1 --no-cpu-baseline --no-config-d --stats-out gpurun_out/bench_d_rehearsal.json > gpurun_out/bench_d_rehearsal.log 2>&1 ;;
    bench_d1) timeout -k 10 900 python bench.py --workload D --steps 2 --warmup 1 --no-cpu-baseline --no-config-d --stats-out gpurun_out/bench_d1.json > gpurun_out/bench_d1.log 2>&1 ;;
    bench_b_rehearsal) MC_BENCH_ONE_GPU=1 timeout -k 10 900 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-config-d --stats-out gpurun_out/bench_b_rehearsal.json > gpurun_out/bench_b_rehearsal.log 2>&1 ;;
    bench_small) timeout -k 10 600 python bench.py --n 20000 --templates 200 --steps 2 --warmup 1 --no-cpu-baseline --no-config-d --stats-out gpurun_out/bench_small.json > gpurun_out/bench_small.log 2>&1 ;;
    bench_align) timeout -k 10 600 python bench.py --n 20000 --templates 200 --id 0.55 --steps 1 --warmup 1 --no-cpu-baseline --no-config-d --stats-out gpurun_out/bench_align.json > gpurun_out/bench_align.log 2>&1 ;;
    bench_nocpu) timeout -k 10 900 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config-d --stats-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 ;;
    bench) timeout -k 10 900 python bench.py --steps 3 --warmup 1 --stats-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 ;;
    prof) timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/prof.log 2>&1 ;;
    pmc_fetch) timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/pmc_fetch.log 2>&1 ;;
    pmc_write) timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/pmc_write.log 2>&1 ;;
    valu) timeout -k 10 120 ./scripts/microbench/valu_peak > gpurun_out/valu_peak.json 2> gpurun_out/valu_peak.err ;;
    accum_prof4) MC_ACCUM_PROFILE=4 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/accum_prof4.log 2>&1 ;;
    accum_prof2) MC_ACCUM_PROFILE=2 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/accum_prof2.log 2>&1 ;;
    accum_prof1) MC_ACCUM_PROFILE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/accum_prof1.log 2>&1 ;;
    *) echo "unknown step $s"; continue ;;
  esac
  rc=$?
  status "$s" "$rc"
  if [ "$s" = pytest ] && [ $rc -eq 1 ]; then continue; fi
  # rocprofv3 on this image segfaults (139) at exit after writing its files: that ends the
  # session too, so give prof / pmc_fetch / pmc_write each a gpurun call of their own (last)
  if [ $rc -ne 0 ]; then exit $rc; fi
done
