#!/bin/bash
# Round-4 call X: multi-rank rehearsal on the final tree (gloo-gpu ranks sharing the one GPU):
# bench.py --verify at 2 / 4 / 8 ranks, distributed sort (look-back passes per rank) and group-by at 8.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04x
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
for g in 2 4 8; do
  CYLON_BENCH_BACKEND=gloo-gpu step bench_multirank_$g 400 python bench.py --gpus $g --rows 40000000 --steps 2 --warmup 1 --verify
done
CYLON_BENCH_BACKEND=gloo-gpu step dist_sort_8 400 python tools/bench_dist.py --gpus 8 --config sort --rows 80000000 --steps 2
CYLON_BENCH_BACKEND=gloo-gpu step dist_groupby_8 400 python tools/bench_dist.py --gpus 8 --config groupby --rows 40000000 --groups 400000 --steps 2
echo done
