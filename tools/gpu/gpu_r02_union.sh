# Union (config 6) after the batched concatenation copy: set-op/merge GPU tests, timing, kernel profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "set or union or merge or concat or list or chunked or interop" > gpurun_out/pytest_union.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/pytest_union.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_suite.py --configs 6 --reps 3 > gpurun_out/bench_cfg6.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_cfg6.log | cut -c1-200
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg6b -o u -- python3 $GRAFT_REPO_ROOT/tools/bench_suite.py --configs 6 --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_cfg6b.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_cfg6b/u_results.db 8 > gpurun_out/prof_cfg6b_summary.txt; cat gpurun_out/prof_cfg6b_summary.txt
