#!/bin/bash
# NW latency-form width A/B on config E9100 (the sampler rounds of 8-12 kb pairs): the default
# (8 waves per pair beyond 1,024 rows) against MC_NW_WAVES forced widths; train phase per width.
#   WIDTHS="default 16 4" bash scripts/nw_width_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${WIDTHS:-default 16}; do
  if [ "$v" = default ]; then env_=(); else env_=(MC_NW_WAVES=$v); fi
  env "${env_[@]}" timeout -k 10 600 python scripts/configs.py ${CFG:-E9100} > gpurun_out/nw_width_$v.log 2>&1 || { echo "rc=$? width $v"; tail -5 gpurun_out/nw_width_$v.log; exit 1; }
  cp gpurun_out/configs_${CFG:-E9100}.json gpurun_out/nw_width_${CFG:-E9100}_$v.json
  python - gpurun_out/nw_width_${CFG:-E9100}_$v.json "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); p = d.get("phases_ms", {})
print("width %s: wall %.3f s train %.1f (search align %.1f, labels %.1f) accumulate %.1f ms" % (
    sys.argv[2], d["wall_s"], p.get("train", 0), p.get("train.nw_search.align", 0), p.get("train.nw_labels", 0), p.get("accumulate", 0)))
PY
done
