#!/bin/bash
# Training / NW A/B on a scripts/configs.py input (default config E9100, whose training is 8-12 kb
# sampler rounds + a label batch): one run per variant, train and accumulation phases.  A
# variant is "default", a width (MC_NW_WAVES=<n>), or VAR=VALUE[,VAR=VALUE...].
#   VARIANTS="default 4 MC_NW_LOOKAHEAD=3" CFG=E9100 bash scripts/nw_width_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-E9100}
for v in ${VARIANTS:-${WIDTHS:-default 4}}; do
  case "$v" in
    default) env_=() ;;
    *=*) env_=(${v//,/ }) ;;
    *) env_=(MC_NW_WAVES=$v) ;;
  esac
  tag=${v//[=,]/_}
  env "${env_[@]}" timeout -k 10 600 python scripts/configs.py $CFG > gpurun_out/nw_ab_$tag.log 2>&1 || { echo "rc=$? variant $v"; tail -5 gpurun_out/nw_ab_$tag.log; exit 1; }
  cp gpurun_out/configs_$CFG.json gpurun_out/nw_ab_${CFG}_$tag.json
  python - gpurun_out/nw_ab_${CFG}_$tag.json "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); p = d.get("phases_ms", {})
print("%s: wall %.3f s train %.1f (search align %.1f, resolve %.1f, labels %.1f) accumulate %.1f ms%s" % (
    sys.argv[2], d["wall_s"], p.get("train", 0), p.get("train.nw_search.align", 0), p.get("train.nw_search.resolve", 0),
    p.get("train.nw_labels", 0), p.get("accumulate", 0),
    "" if "partition_equals_reference" not in d else " partition==ref %s" % d["partition_equals_reference"]))
PY
done
