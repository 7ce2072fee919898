#!/bin/bash
# Round-4 call F: composite-key proxy joins (tests + 100M/1B join-type timings), 2/4/8-rank gloo-gpu
# rehearsal (bench --verify, distributed group-by and sort), k_rg_agg diag under the exact-slot
# tables, and self-RCCL overlap variants (8 chunks; more RCCL p2p channels).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_new 300 python -u -m pytest tests/test_gpu_radix_joins.py -x -v --timeout 200 --timeout-method thread
step jt_100m 300 python tools/join_types_probe.py 100000000 3 inner,left,right,outer,inner2,left2
step jt_1b 600 python tools/join_types_probe.py 1000000000 2 inner,left,outer,inner2
for g in 2 4 8; do
  CYLON_BENCH_BACKEND=gloo-gpu step bench_multirank_$g 400 python bench.py --gpus $g --rows 40000000 --steps 2 --warmup 1 --verify
done
CYLON_BENCH_BACKEND=gloo-gpu step dist_groupby_8 300 python tools/bench_dist.py --gpus 8 --config groupby --rows 40000000 --groups 400000 --steps 2
CYLON_BENCH_BACKEND=gloo-gpu step dist_sort_8 300 python tools/bench_dist.py --gpus 8 --config sort --rows 80000000 --steps 2
AMD_SERIALIZE_KERNEL=3 CYLON_RG_WIDE=1 step rg_wide_plain 120 python tools/diag_groupby_xt.py 1 3000000 2
CYLON_SHUFFLE_CHUNKS=8 CYLON_SHUFFLE_SELF_RCCL=1 step selfrccl_k8 300 python bench.py --force-shuffle --rows 500000000 --steps 10 --warmup 3
CYLON_SHUFFLE_CHUNKS=4 CYLON_SHUFFLE_SELF_RCCL=1 NCCL_MIN_P2P_NCHANNELS=32 step selfrccl_k4_ch32 300 python bench.py --force-shuffle --rows 500000000 --steps 10 --warmup 3
CYLON_SHUFFLE_CHUNKS=8 CYLON_SHUFFLE_SELF_RCCL=1 NCCL_MIN_P2P_NCHANNELS=32 step selfrccl_k8_ch32 300 python bench.py --force-shuffle --rows 500000000 --steps 10 --warmup 3
CYLON_SHUFFLE_CHUNKS=8 CYLON_SHUFFLE_SELF_RCCL=1 step prof_selfrccl_k8 300 rocprofv3 --kernel-trace --stats -d $O/prof_selfrccl_k8 -o k8 -- python3 bench.py --force-shuffle --rows 500000000 --steps 1 --warmup 1 --no-phases
CYLON_SHUFFLE_CHUNKS=4 CYLON_SHUFFLE_SELF_RCCL=1 NCCL_MIN_P2P_NCHANNELS=32 step prof_selfrccl_ch32 300 rocprofv3 --kernel-trace --stats -d $O/prof_selfrccl_ch32 -o ch32 -- python3 bench.py --force-shuffle --rows 500000000 --steps 1 --warmup 1 --no-phases
step bench_forced_default 300 python bench.py --force-shuffle --steps 20 --warmup 5
echo done
