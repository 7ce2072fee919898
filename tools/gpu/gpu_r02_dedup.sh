# Set-op dedup reuses the slots claimed in phase 1: set-op tests + union config.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_kernels.py tests/test_gpu_multirank.py -k "set or union or unique or distinct or subtract or intersect" > gpurun_out/dd_tests.log 2>&1 || { tail -40 gpurun_out/dd_tests.log; exit 1; }
tail -1 gpurun_out/dd_tests.log
timeout -k 10 600 python -u tools/bench_suite.py --configs 6 --reps 3 > gpurun_out/dd_suite.log 2>&1 || exit 1
grep '^{' gpurun_out/dd_suite.log | cut -c1-300
