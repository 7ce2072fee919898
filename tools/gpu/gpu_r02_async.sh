# Async exchange path on the device + native bootstrap example + new sort dtype cases, then an
# overlap kernel trace of the chunked join under the asynchronous delay transport.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_kernels.py -k "async or radix_row_sort or chunked" > gpurun_out/pytest_async.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_async.log; tail -5 gpurun_out/pytest_async.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./examples/cpp/bin/async_overlap_example 4000000 4 3000 29655 > gpurun_out/async_overlap.log 2>&1 || exit 1
cat gpurun_out/async_overlap.log | grep rank
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_async -o async -- $GRAFT_REPO_ROOT/examples/cpp/bin/async_overlap_example 4000000 4 3000 29656 > $GRAFT_REPO_ROOT/gpurun_out/prof_async.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/overlap_report.py gpurun_out/prof_async/async_results.db > gpurun_out/async_overlap_report.txt; tail -20 gpurun_out/async_overlap_report.txt
