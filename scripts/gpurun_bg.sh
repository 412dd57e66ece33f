#!/bin/bash
# Submit one gpurun call from this container, waiting while the pool has no free box or slot
# (gpurun exit code 3: nothing ran, nothing charged).  Any other outcome -- success or a
# failure of the command itself -- ends it: a failing GPU step is never re-run.
#   scripts/gpurun_bg.sh OUT.txt TIMEOUT 'command'
out=$1 lim=$2 cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  grep -q "no free box\|slot(s) on this pod are busy\|stopped responding while being prepared\|backing off" "$out" || break
  sleep 90
done
echo "[gpurun_bg] rc=$rc" >> "$out"
