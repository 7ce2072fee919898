# Final validation of the session-3 tree: full GPU suite, smoke, default bench, join kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final4.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu_final4.log; grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu_final4.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final4.log 2>&1 || exit 1
tail -1 gpurun_out/smoke_final4.log
timeout -k 10 600 python bench.py > gpurun_out/bench_final4.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_final4.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --verify > gpurun_out/bench_verify4.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_verify4.log | cut -c1-400
