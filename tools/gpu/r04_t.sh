#!/bin/bash
# Round-4 call T: look-back walk after the key staging (predecessors get the staging time to publish):
# look-back tests, sort tests, interleaved config-5 A/B against CYLON_SORT_LOOKBACK=0, kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04t
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_lb 240 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 100 --timeout-method thread -k "lookback"
grep -q "pytest_lb rc=0" $O/steps.txt || exit 1
step pytest_sort 500 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "sort"
step suite5_a 300 python tools/bench_suite.py --configs 5 --reps 3
CYLON_SORT_LOOKBACK=0 step suite5_x 300 python tools/bench_suite.py --configs 5 --reps 3
step suite5_b 300 python tools/bench_suite.py --configs 5 --reps 3
step prof_sort 300 rocprofv3 --kernel-trace --stats -d $O/prof_sort -o sort -- python3 tools/bench_suite.py --configs 5 --reps 1
echo done
