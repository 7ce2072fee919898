set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_join1b -o join -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_join1b.log 2>&1
echo "prof exit $?"
cd $GRAFT_REPO_ROOT
find gpurun_out/prof_join1b -name "*stats*" | head
