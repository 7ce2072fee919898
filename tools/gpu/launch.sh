#!/bin/bash
# launch.sh <script> [log]: run one GPU call script through gpurun, waiting (up to ~40 min) while the
# pool reports no free box / slot (gpurun exit 3: nothing ran, nothing charged).  Any other outcome
# -- including a failure of the script itself -- ends the loop: a failing GPU step is never retried.
S=$1
LOG=${2:-/tmp/gpurun_last.log}
for i in $(seq 1 16); do
  timeout 1700 /usr/local/graft/bin/gpurun --timeout 1200 -- "bash $S" > "$LOG" 2>&1
  rc=$?
  [ "$rc" -eq 3 ] || break
  sleep 150
done
echo "gpurun rc=$rc"
tail -3 "$LOG"
