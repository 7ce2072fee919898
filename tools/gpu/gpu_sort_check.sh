# GPU suite + smoke + table-sort config + headline bench after a sort-path change.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python tools/bench_suite.py --configs 5 > gpurun_out/bench_cfg5.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_cfg5.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_default.log
