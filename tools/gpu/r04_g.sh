#!/bin/bash
# Round-4 call G: slot-mode join partitions (tests, A/B, verify), full GPU suite (composite-key proxies, 8 default chunks), headline bench, the
# timed-vs-traced gap diagnosis (allocator retries; per-step sync), the FULL OUTER kernel trace,
# then the PMC pass set of the headline join kernels.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_slot 240 python -u -m pytest tests/test_gpu_radix_joins.py -x -v --timeout 120 --timeout-method thread -k "slot"
step bench_1 200 python bench.py --steps 20 --warmup 5
CYLON_RJ_SLOT=0 step bench_1_noslot 200 python bench.py --steps 20 --warmup 5
step bench_1_verify 200 python bench.py --steps 3 --warmup 1 --verify
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_forced_default 300 python bench.py --force-shuffle --steps 20 --warmup 5
CYLON_SHUFFLE_CHUNKS=4 step bench_forced_k4 300 python bench.py --force-shuffle --steps 10 --warmup 3
CYLON_SHUFFLE_CHUNKS=4 CYLON_SHUFFLE_SELF_RCCL=1 NCCL_MIN_P2P_NCHANNELS=32 step gap_ch32 300 python bench.py --force-shuffle --rows 500000000 --steps 10 --warmup 3
CYLON_SHUFFLE_CHUNKS=4 CYLON_SHUFFLE_SELF_RCCL=1 NCCL_MIN_P2P_NCHANNELS=32 step gap_ch32_sync 300 python bench.py --force-shuffle --rows 500000000 --steps 10 --warmup 3 --sync-steps
CYLON_SHUFFLE_SELF_RCCL=1 step selfrccl_default 300 python bench.py --force-shuffle --rows 500000000 --steps 10 --warmup 3
step prof_outer 300 rocprofv3 --kernel-trace --stats -d $O/prof_outer -o outer -- python3 tools/join_types_probe.py 1000000000 1 inner,outer
step pmc 900 bash tools/gpu/r04_pmc.sh head
echo done
