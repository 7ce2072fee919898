#!/bin/bash
# Round-4 first call: baselines before the distributed-join / outer-join work, then the k_rg_agg diagnosis.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --force-shuffle --steps 5 --warmup 2 > $O/bench_forced.json 2> $O/bench_forced.err
timeout -k 10 300 python tools/join_types_probe.py 100000000 3 inner,left,right,outer,inner2 > $O/jt_100m.jsonl 2> $O/jt_100m.err
timeout -k 10 400 python tools/join_types_probe.py 1000000000 2 inner,left,outer,inner2 > $O/jt_1b.jsonl 2> $O/jt_1b.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_forced -o forced -- python3 bench.py --force-shuffle --steps 1 --warmup 1 > $O/prof_forced.log 2>&1
# k_rg_agg diagnosis: the round-3 faulting shape (two accumulators in the <3, 2048> table), bounds-checked first
AMD_SERIALIZE_KERNEL=3 CYLON_RG_WIDE=1 CYLON_RG_DEBUG=1 timeout -k 10 120 python tools/diag_groupby_xt.py 1 3000000 2 > $O/rg_wide_debug.txt 2>&1
AMD_SERIALIZE_KERNEL=3 CYLON_RG_WIDE=1 timeout -k 10 120 python tools/diag_groupby_xt.py 1 3000000 2 > $O/rg_wide_plain.txt 2>&1
echo done
