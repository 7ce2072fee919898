# GPU validation: radix-join tests first, full GPU suite, 1B bench, kernel profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }   # 1 = test failures (no fault): keep going
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -k radix > gpurun_out/pytest_radix.log 2>&1
rc=$?; echo "radix pytest exit $rc" >> gpurun_out/pytest_radix.log; tail -15 gpurun_out/pytest_radix.log
ok $rc || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -8 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_1b.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_1b.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_join1b -o join -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_join1b.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_join1b/join_results.db 30 > gpurun_out/prof_join1b_summary.txt; cat gpurun_out/prof_join1b_summary.txt
