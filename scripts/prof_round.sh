#!/bin/bash
# rocprofv3 evidence per configuration (one step per argument, each under its own time limit;
# the first failing step ends the session).  Inputs are generated first (CPU only):
#   gen_b gen_c gen_d gen_e                       FASTA of config B / C20k / D1M / E9100
#   stats_X                                       --kernel-trace --stats of bin/meshclust on X
#   pmc_sq_X                                      8 SQ counters (VALU / LDS / busy) on X
#   fetch_X write_X                               TCC FETCH_SIZE / WRITE_SIZE passes on X
# X in b c d e.  The accumulation kernel takes a plain launch under the profiler
# (MC_ACCUM_PLAIN_LAUNCH): a cooperative launch faults rocprofv3's exit handler
# (profiles/r02_rocprof_exit/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out /tmp/mc_cfg
export TMPDIR=/tmp MC_ACCUM_PLAIN_LAUNCH=1
BIN=./meshclust_amd/bin/meshclust
declare -A FA=([b]=/tmp/mc_cfg/B100k.fa [c]=/tmp/mc_cfg/C20k.fa [d]=/tmp/mc_cfg/D1M.fa [e]=/tmp/mc_cfg/E9100.fa)
declare -A FL=([b]="--id 0.90" [c]="--id 0.55 --align" [d]="--id 0.90" [e]="--id 0.80")
gen() {  # name generator-args...
  python - "$@" <<'PY'
import os, sys
sys.path.insert(0, ".")
from meshclust_amd import synth
out, kind, *a = sys.argv[1:]
if not os.path.exists(out):
    if kind == "reads":
        synth.generate(out + ".tmp", *[int(a[0]), int(a[1]), int(a[2]), float(a[3]), int(a[4])])
    else:
        synth.write_fasta(out + ".tmp", synth.families(int(a[0]), int(a[1]), int(a[2]), int(a[3]), float(a[4]), float(a[5]), int(a[6])))
    os.replace(out + ".tmp", out)
print("input", out, os.path.getsize(out))
PY
}
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES"
for s in "$@"; do
  x=${s##*_}
  case $s in
    gen_b) gen ${FA[b]} reads 100000 1000 1000 0.03 41 ;;
    gen_c) gen ${FA[c]} reads 20000 1000 200 0.03 41 ;;
    gen_d) gen ${FA[d]} reads 1000000 1000 10000 0.03 51 ;;
    gen_e) gen ${FA[e]} families 70 130 8000 12000 0.05 0.15 61 ;;
    stats_*) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_$x -o run -- \
               $BIN ${FA[$x]} ${FL[$x]} --threads 16 --output /tmp/mc_cfg/o_$x.clstr --stats-json gpurun_out/stats_$x.json --quiet \
               > gpurun_out/stats_$x.log 2>&1 ;;
    pmc_sq_*) timeout -k 10 300 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d gpurun_out/pmc_sq_$x -o run -- \
               $BIN ${FA[$x]} ${FL[$x]} --threads 16 --output /tmp/mc_cfg/o_$x.clstr --quiet > gpurun_out/pmc_sq_$x.log 2>&1 ;;
    fetch_*) timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/fetch_$x -o run -- \
               $BIN ${FA[$x]} ${FL[$x]} --threads 16 --output /tmp/mc_cfg/o_$x.clstr --quiet > gpurun_out/fetch_$x.log 2>&1 ;;
    write_*) timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/write_$x -o run -- \
               $BIN ${FA[$x]} ${FL[$x]} --threads 16 --output /tmp/mc_cfg/o_$x.clstr --quiet > gpurun_out/write_$x.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "$s rc=$rc t=$(date +%s)" | tee -a gpurun_out/prof_status.txt
  [ $rc -eq 0 ] || exit $rc
done
