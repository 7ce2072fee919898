#!/bin/bash
# Round-4 call AC: last check of the final tree: bench at the driver's settings, --verify, 2-rank gloo-gpu verify.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04ac
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step bench_1 200 python bench.py --steps 20 --warmup 5
step bench_verify 200 python bench.py --steps 3 --warmup 1 --verify
CYLON_BENCH_BACKEND=gloo-gpu step bench_multirank_2 400 python bench.py --gpus 2 --rows 40000000 --steps 2 --warmup 1 --verify
echo done
