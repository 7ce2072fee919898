#!/bin/bash
# With the XCD-tile schedule: classic (one block per CU, next-column prefetch) vs lean (two blocks per CU)
# pass kernel for the 4-column join passes, interleaved.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03lean2
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/classic_$i.json 2> $O/classic_$i.err
  CYLON_RP_KERNEL=lean timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/lean_$i.json 2> $O/lean_$i.err
done
echo done
