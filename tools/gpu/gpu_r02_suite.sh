# Full GPU suite + smoke + default bench on the current tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_default.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_default.log
