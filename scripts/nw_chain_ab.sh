#!/bin/bash
# NW parity (every chain form) + config E9100 / C20k under each row-block hand-off setting;
# every GPU step under its own limit, the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-nwc}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q \
  -k "${K:-nw or E91}" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-1 r16 2 0}; do
  case $v in
    *=*) env="${v//,/ }";;
    r16) env="MC_NW_CHAIN_R=16";;
    r8) env="MC_NW_CHAIN_R=8";;
    2r8) env="MC_NW_CHAIN=2 MC_NW_CHAIN_R=8";;
    *) env="MC_NW_CHAIN=$v";;
  esac
  env $env timeout -k 10 300 python scripts/configs.py ${CFGS:-E9100} > gpurun_out/${TAG}_cfg_${v//[=,]/_}.log 2>&1 || exit 1
done
python - <<'PY'
import glob, json, os
tag = os.environ.get("TAG", "nwc")
for f in sorted(glob.glob("gpurun_out/%s_cfg_*.log" % tag)):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); p = d.get("phases_ms") or {}
            print(f, d["config"], d["wall_s"], {k: p.get(k) for k in ("train.nw_search.align", "train.nw_labels", "train", "accumulate.window")})
PY
