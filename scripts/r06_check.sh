#!/bin/bash
# Round-6 GPU check.  Steps (names in $STEPS, run in order, each under its own time limit; the
# first failing step ends the call):
#   pytest     pytest -m gpu selection (-k "$K", files $FILES)
#   bench      bench.py config B (+ config D in extra.config_d), no reference baseline
#   benchfull  bench.py with its defaults (the driver's command: reference baseline included)
#   rehearsal  two ranks on the one GPU (MC_BENCH_ONE_GPU=1 --gpus 2), config B + config D
#   prof1      MC_ACCUM_PROFILE=1 bench (controller phase timers)
#   prof4      MC_ACCUM_PROFILE=4 bench (per-worker step trace)
#   configs    scripts/configs.py $CONFIGS
#   calib      FETCH_SIZE of the known-byte-count reads of scripts/microbench/fetch_calib
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06}
run() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -n 30 "gpurun_out/${TAG}_$name.log"; exit $rc; }
}
for s in ${STEPS:-pytest bench}; do
  case $s in
    pytest) run pytest 1100 python -u -m pytest ${FILES:-tests} -m gpu -x -v -k "${K:-gpu}" --timeout 600 \
              --timeout-method thread -p no:cacheprovider
            tail -n 2 gpurun_out/${TAG}_pytest.log ;;
    bench) run bench 600 python bench.py --steps ${BSTEPS:-10} --warmup 2 --no-cpu-baseline --stats-out gpurun_out/${TAG}_bench.json ;;
    benchfull) run benchfull 900 python bench.py ;;
    rehearsal) MC_BENCH_ONE_GPU=1 run rehearsal 900 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline ;;
    prof1) MC_ACCUM_PROFILE=1 run prof1 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config-d ;;
    prof4) MC_ACCUM_PROFILE=4 run prof4 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-d ;;
    configs) run configs 900 python scripts/configs.py $CONFIGS ;;
    calib) run calib 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_calib -o run \
             -- ./scripts/microbench/fetch_calib ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
python - <<'PY'
import glob, json, os
tag = os.environ.get("TAG", "r06")
for f in sorted(glob.glob("gpurun_out/%s_*.log" % tag)):
    l = [x for x in open(f) if x.startswith("{")]
    if not l:
        continue
    d = json.loads(l[-1])
    e = d["extra"]
    r = d["roofline"] or {}
    print(f, "value %.0f ms/step %.2f us/step %s frac %s" % (d["value"], d["ms_per_step"], r.get("us_per_step"), r.get("frac")),
          "train %.2f" % e["host_phases_ms"].get("train", 0), json.dumps(e.get("step_split_ms")))
    cd = e.get("config_d")
    if cd:
        print("   config_d: value %.0f ms/step %.1f path %s roof %s" % (cd["value"], cd["ms_per_step"], cd["accum_path"],
              (cd["roofline"] or {}).get("frac")))
PY
grep -h "^\[accum" gpurun_out/${TAG}_prof1.log 2>/dev/null | head -n 6
grep -h "trace4" gpurun_out/${TAG}_prof4.log 2>/dev/null | head -n 2
exit 0
