#!/bin/bash
# Kernel trace of the config E9100 run (chained row blocks on, then off): per-dispatch grid and
# duration of every NW launch, for the latency-form analysis in DESIGN.md §4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-E9100}
FA=$(python - <<PY
import sys; sys.path.insert(0, "scripts"); import configs, os, tempfile
d = os.path.join(tempfile.gettempdir(), "mc_cfg"); os.makedirs(d, exist_ok=True)
print(configs.make_input(configs.CONFIGS["$CFG"][0], os.path.join(d, "$CFG.fa")))
PY
) || exit 1
FLAGS=$(python -c "import sys; sys.path.insert(0, 'scripts'); import configs; print(' '.join(configs.CONFIGS['$CFG'][1]))")
for ch in ${CHAINS:-1 0}; do
  export MC_NW_CHAIN=$ch
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/nwprof_$ch -o run -- \
    meshclust_amd/bin/meshclust "$FA" $FLAGS --threads 16 --output /tmp/nwp.clstr --stats-json gpurun_out/nwprof_$ch.stats.json --quiet \
    > gpurun_out/nwprof_$ch.log 2>&1 || exit 1
done
