# Full GPU validation: pytest -m gpu, smoke, 1B bench, kernel profile, secondary configs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -8 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_default.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_join1b -o join -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_join1b.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_join1b/join_results.db 30 > gpurun_out/prof_join1b_summary.txt; head -12 gpurun_out/prof_join1b_summary.txt
timeout -k 10 900 python tools/bench_suite.py > gpurun_out/bench_suite.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/bench_suite.log
