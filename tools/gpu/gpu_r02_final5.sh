# Secondary configs + headline kernel trace on the final session-3 tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/bench_suite.py --configs 2,4,5,6,7 --reps 3 > gpurun_out/bench_suite_final5.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_suite_final5.log | cut -c1-170
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_final5 -o join -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-phases > $GRAFT_REPO_ROOT/gpurun_out/prof_final5.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_final5/join_results.db 12 > gpurun_out/prof_final5_summary.txt; head -8 gpurun_out/prof_final5_summary.txt
