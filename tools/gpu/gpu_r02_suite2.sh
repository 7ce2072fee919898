# GPU suite + secondary configs (union / group-by / sort / join 100M) after the round-2 changes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/bench_suite.py --configs 2,4,5,6 --reps 3 > gpurun_out/bench_suite.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_suite.log | cut -c1-260
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg6 -o u -- python3 $GRAFT_REPO_ROOT/tools/bench_suite.py --configs 6 --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_cfg6.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_cfg6/u_results.db 14 > gpurun_out/prof_cfg6_summary.txt; cat gpurun_out/prof_cfg6_summary.txt
timeout -k 10 600 python -u tools/rank_sim.py --sort 2000000000 2 4 8 > gpurun_out/rank_sim_sort.log 2>&1 || exit 1
grep SORT gpurun_out/rank_sim_sort.log
