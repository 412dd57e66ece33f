#!/bin/bash
# Round-5 multi-rank session on the one-GPU box: the distributed GPU tests (ranks sharing the
# GPU through CU partitions, no environment override), then the two-rank rehearsal bench lines
# (MC_BENCH_ONE_GPU=1: both ranks on GPU 0, each on its CU partition, gloo all-gathers) for
# config B and D, each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 1200 python -u -m pytest tests/test_distributed.py -m gpu -x -v --timeout 900 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/multi_pytest.log 2>&1
  rc=$?; tail -n 25 gpurun_out/multi_pytest.log | grep -E "PASS|FAIL|ERROR|passed|failed|skipped" | tail -n 30; [ $rc -eq 0 ] || exit $rc
fi
MC_BENCH_ONE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-config-d \
  --stats-out gpurun_out/multi_b2_stats.json > gpurun_out/multi_b2.log 2>&1 || { echo "b2 rc=$?"; tail -n 30 gpurun_out/multi_b2.log; exit 1; }
if [ -n "${D:-}" ]; then
  MC_BENCH_ONE_GPU=1 timeout -k 10 900 python bench.py --gpus 2 --workload D --steps 2 --warmup 1 --no-cpu-baseline --no-config-d \
    --stats-out gpurun_out/multi_d2_stats.json > gpurun_out/multi_d2.log 2>&1 || { echo "d2 rc=$?"; tail -n 30 gpurun_out/multi_d2.log; exit 1; }
fi
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/multi_*2.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l:
        continue
    d = json.loads(l[-1])
    e = d["extra"]
    print(f, "value %.0f ms/step %.2f accum %s" % (d["value"], d["ms_per_step"], e.get("accum_path")))
    print("  phases", json.dumps({k: round(v, 2) for k, v in e["host_phases_ms"].items() if not k.startswith("comm.")}))
    print("  comm", json.dumps(e.get("comm_ms_per_step")))
PY
