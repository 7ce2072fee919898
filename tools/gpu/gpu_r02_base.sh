# Round-2 baseline on the rebuilt tree: GPU suite, smoke, default bench, verified 1B bench, kernel profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -8 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_default.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --verify > gpurun_out/bench_verify.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_verify.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_join1b -o join -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-phases > $GRAFT_REPO_ROOT/gpurun_out/prof_join1b.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_join1b/join_results.db 30 > gpurun_out/prof_join1b_summary.txt; head -14 gpurun_out/prof_join1b_summary.txt
