#!/bin/bash
# Round-4 call P: sort digits of image - min (7 x 9-bit digits for keys spanning 63 bits): sort tests,
# config-5 A/B against CYLON_SORT_SUB_MIN=0, kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04p
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_sort 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "sort"
step suite5 300 python tools/bench_suite.py --configs 5 --reps 3
CYLON_SORT_SUB_MIN=0 step suite5_nosub 300 python tools/bench_suite.py --configs 5 --reps 3
step prof_sort 300 rocprofv3 --kernel-trace --stats -d $O/prof_sort -o sort -- python3 tools/bench_suite.py --configs 5 --reps 1
echo done
