#!/bin/bash
# Partition bits with the XCD-tile passes: 18 (9+9, default), 19 (10+9), 20 (10+10) -- pass and write times.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03bits
mkdir -p $O
for x in 0 1 2 0; do
  CYLON_RJ_EXTRA_BITS=$x timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/bits_$x.json 2> $O/bits_$x.err
done
CYLON_RJ_EXTRA_BITS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof20 -o j -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof20.log 2>&1
echo done
