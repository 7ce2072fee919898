set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_1b.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_1b.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_join1b -o join -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_join1b.log 2>&1
echo "prof exit $?"
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_join1b/join_results.db 30 > gpurun_out/prof_join1b_summary.txt; cat gpurun_out/prof_join1b_summary.txt
