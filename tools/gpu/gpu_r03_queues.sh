#!/bin/bash
# Which hardware queue the RCCL stream lands on (forced world-1 shuffle) and whether its
# all-to-all kernels overlap the join kernels, for stream-priority / queue-count settings.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03q
mkdir -p $O
run() {
  local tag=$1; shift
  ( export "$@"; timeout -k 10 200 rocprofv3 --kernel-trace -d $O/$tag -o $tag -- python3 bench.py --rows 200000000 --steps 2 --warmup 1 --force-shuffle --no-phases > $O/$tag.log 2>&1 )
  python3 tools/queue_map.py $(ls $O/$tag/*_results.db $O/$tag/*/*_results.db 2>/dev/null | head -1) >> $O/summary.txt
  echo "== $tag" >> $O/summary.txt
}
run default A=1
run highprio TORCH_NCCL_HIGH_PRIORITY=1
run hwq8 GPU_MAX_HW_QUEUES=8
echo done
