# 1024-thread passes whenever ranking is LDS-atomic: tests + secondary configs + headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_thr.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu_thr.log; grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu_thr.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/bench_suite.py --configs 2,4,5,6 --reps 3 > gpurun_out/bench_suite_thr.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_suite_thr.log | cut -c1-170
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_thr.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_thr.log | cut -c1-300
