#!/bin/bash
# Round-5 GPU check: a pytest selection (-k "$K", files $FILES), then bench lines for config B
# (and D when $D is set); every GPU step under its own limit, the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-chk}
if [ -n "${K:-}" ]; then
  timeout -k 10 900 python -u -m pytest ${FILES:-tests} -m gpu -x -q -k "$K" --timeout 600 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -n 3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${NOB:-}" ]; then
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-config-d > gpurun_out/${TAG}_bench_b.log 2>&1 || exit 1
fi
if [ -n "${D:-}" ]; then
  timeout -k 10 600 python bench.py --workload D --steps 2 --warmup 1 --no-cpu-baseline --no-config-d > gpurun_out/${TAG}_bench_d.log 2>&1 || exit 1
fi
if [ -n "${CONFIGS:-}" ]; then
  timeout -k 10 900 python scripts/configs.py $CONFIGS > gpurun_out/${TAG}_configs.log 2>&1 || exit 1
fi
python - <<'PY'
import glob, json, os
tag = os.environ.get("TAG", "chk")
for f in sorted(glob.glob("gpurun_out/%s_bench_*.log" % tag)):
    l = [x for x in open(f) if x.startswith("{")]
    if not l:
        continue
    d = json.loads(l[-1])
    e = d["extra"]
    k1 = e["kernel_rooflines"].get("kmer_kernel", {})
    print(f, "value %.0f ms/step %.2f us/step %s kmer_us %s frac %s" % (d["value"], d["ms_per_step"], d["roofline"]["us_per_step"],
          k1.get("avg_launch_us"), k1.get("frac")), json.dumps(e["device_ms_per_step"]))
PY
