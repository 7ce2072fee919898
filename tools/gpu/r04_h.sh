#!/bin/bash
# Round-4 call H: slot mode v2 (static per-XCD tile dealing, early cursor atomics; 18-bit outer
# joins), A/B against the exact LSD passes, join types, kernel trace of the headline join.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04h
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_slot 300 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "slot or ranking_guard or outer or composite"
step bench_1 200 python bench.py --steps 20 --warmup 5
CYLON_RJ_SLOT=0 step bench_1_noslot 200 python bench.py --steps 20 --warmup 5
step bench_1_verify 200 python bench.py --steps 3 --warmup 1 --verify
step jt_1b 600 python tools/join_types_probe.py 1000000000 2 inner,left,outer,inner2
step prof_head 300 rocprofv3 --kernel-trace --stats -d $O/prof_head -o head -- python3 bench.py --steps 2 --warmup 1 --no-phases
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo done
