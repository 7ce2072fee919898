# Sort: first pass images raw 8-byte integer keys (no image write): tests + config 5 + trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_ops.py tests/test_properties.py -k "sort or stable or gpu_" > gpurun_out/raw_tests.log 2>&1 || { tail -40 gpurun_out/raw_tests.log; exit 1; }
tail -1 gpurun_out/raw_tests.log
timeout -k 10 600 python -u tools/bench_suite.py --configs 5 --reps 3 > gpurun_out/raw_suite.log 2>&1 || exit 1
grep '^{' gpurun_out/raw_suite.log | cut -c1-220
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_raw5 -o s -- python3 $GRAFT_REPO_ROOT/tools/bench_suite.py --configs 5 --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_raw5.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_raw5/s_results.db 10 > gpurun_out/prof_raw5_summary.txt; cat gpurun_out/prof_raw5_summary.txt
