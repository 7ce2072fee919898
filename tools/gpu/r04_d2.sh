#!/bin/bash
# Round-4 call D2: overlap trace of the forced RCCL path, join-type timings, 8-rank gloo-gpu
# rehearsal (bench --verify, distributed group-by and sort), then the k_rg_agg diagnosis.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
CYLON_SHUFFLE_CHUNKS=4 CYLON_SHUFFLE_SELF_RCCL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_selfrccl -o selfrccl -- python3 bench.py --force-shuffle --rows 500000000 --steps 1 --warmup 1 --no-phases > $O/prof_selfrccl.log 2>&1
CYLON_SHUFFLE_CHUNKS=4 CYLON_SHUFFLE_SELF_RCCL=1 timeout -k 10 300 python bench.py --force-shuffle --rows 500000000 --steps 10 --warmup 3 > $O/bench_forced_k4_selfrccl_500m.json 2> $O/bench_forced_k4_selfrccl.err
CYLON_SHUFFLE_CHUNKS=4 timeout -k 10 300 python bench.py --force-shuffle --steps 10 --warmup 3 > $O/bench_forced_k4.json 2> $O/bench_forced_k4.err
CYLON_SHUFFLE_CHUNKS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_k4 -o k4 -- python3 bench.py --force-shuffle --steps 1 --warmup 1 --no-phases > $O/prof_k4.log 2>&1
timeout -k 10 300 python tools/join_types_probe.py 100000000 3 inner,left,right,outer,inner2 > $O/jt_100m.jsonl 2> $O/jt_100m.err
timeout -k 10 500 python tools/join_types_probe.py 1000000000 2 inner,left,outer,inner2 > $O/jt_1b.jsonl 2> $O/jt_1b.err
CYLON_BENCH_BACKEND=gloo-gpu timeout -k 10 400 python bench.py --gpus 8 --rows 40000000 --steps 2 --warmup 1 --verify > $O/bench_multirank_8.json 2> $O/bench_multirank_8.err
CYLON_BENCH_BACKEND=gloo-gpu timeout -k 10 300 python tools/bench_dist.py --gpus 8 --config groupby --rows 40000000 --groups 400000 --steps 2 > $O/dist_groupby_8.json 2> $O/dist_groupby_8.err
CYLON_BENCH_BACKEND=gloo-gpu timeout -k 10 300 python tools/bench_dist.py --gpus 8 --config sort --rows 80000000 --steps 2 > $O/dist_sort_8.json 2> $O/dist_sort_8.err
AMD_SERIALIZE_KERNEL=3 CYLON_RG_WIDE=1 CYLON_RG_DEBUG=1 timeout -k 10 120 python tools/diag_groupby_xt.py 1 3000000 2 > $O/rg_wide_debug.txt 2>&1
AMD_SERIALIZE_KERNEL=3 CYLON_RG_WIDE=1 timeout -k 10 120 python tools/diag_groupby_xt.py 1 3000000 2 > $O/rg_wide_plain.txt 2>&1
echo done
