# Kernel trace of the nullable 200M x 200M radix join.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_null -o n -- python3 $GRAFT_REPO_ROOT/tools/nullable_probe.py --only-nullable > $GRAFT_REPO_ROOT/gpurun_out/prof_null.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_null/n_results.db 14 > gpurun_out/prof_null_summary.txt; cat gpurun_out/prof_null_summary.txt
