# Kernel traces of group-by (config 4) and union (config 6) on the final tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_g4 -o g -- python3 $GRAFT_REPO_ROOT/tools/bench_suite.py --configs 4 --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_g4.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_g4/g_results.db 12 > gpurun_out/prof_g4_summary.txt; cat gpurun_out/prof_g4_summary.txt
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_u6 -o u -- python3 $GRAFT_REPO_ROOT/tools/bench_suite.py --configs 6 --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_u6.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_u6/u_results.db 12 > gpurun_out/prof_u6_summary.txt; cat gpurun_out/prof_u6_summary.txt
