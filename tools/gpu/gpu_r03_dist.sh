#!/bin/bash
# Multi-rank rehearsal of bench.py on the one-GPU box: 2 and 4 ranks sharing cuda:0 with gloo
# collectives (tables in HBM, every radix pass on the XCD-tile schedule), --verify on each.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03dist
mkdir -p $O
export CYLON_BENCH_BACKEND=gloo-gpu
timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --rows 40000000 --verify > $O/w2.json 2> $O/w2.err
timeout -k 10 300 python bench.py --gpus 4 --steps 3 --warmup 1 --rows 40000000 --verify > $O/w4.json 2> $O/w4.err
echo done
