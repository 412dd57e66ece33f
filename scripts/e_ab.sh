cd "${GRAFT_REPO_ROOT}"
for v in ${VARIANTS:-base}; do
  envs=(); [ "$v" != base ] && envs=(${v//,/ })
  env "${envs[@]}" timeout -k 10 200 python scripts/configs.py E9100 > gpurun_out/e_ab.txt 2>&1 || { tail gpurun_out/e_ab.txt; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/e_ab.txt') if l.startswith('{')][-1]); p=d['phases_ms']; print('$v', d['wall_s'], p['train'], p['train.nw_search'], p['train.nw_labels'], d['nw_pairs'], d['clusters'], p['accumulate'])"
done
