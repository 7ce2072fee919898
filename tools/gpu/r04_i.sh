#!/bin/bash
# Round-4 call I: histogram-free FIRST join pass ((bucket, XCD) slots) + sort next-digit arrays:
# targeted tests first, then A/B benches, the sort config, the full suite, a kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_targeted 400 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -k "slot or ranking_guard or outer or composite or sort"
step bench_1 200 python bench.py --steps 20 --warmup 5
step bench_1_verify 200 python bench.py --steps 3 --warmup 1 --verify
CYLON_RJ_SLOT=0 step bench_1_noslot 200 python bench.py --steps 20 --warmup 5
step suite5 400 python tools/bench_suite.py --configs 5 --reps 3
CYLON_SORT_NEXT_DIGITS=0 step suite5_nond 400 python tools/bench_suite.py --configs 5 --reps 3
step jt_1b 600 python tools/join_types_probe.py 1000000000 2 inner,left,outer,inner2
step prof_head 300 rocprofv3 --kernel-trace --stats -d $O/prof_head -o head -- python3 bench.py --steps 2 --warmup 1 --no-phases
step prof_sort 300 rocprofv3 --kernel-trace --stats -d $O/prof_sort -o sort -- python3 tools/bench_suite.py --configs 5 --reps 1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo done
