# LDS-only barriers + branch-free loads in k_rows_pass: correctness, stamps, join + sort timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_kernels.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ldsbar.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -1 gpurun_out/pytest_ldsbar.log
[ $rc -eq 0 ] || exit $rc
CYLON_RP_STAMPS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-phases > gpurun_out/stamps_join2.log 2>&1 || exit 1
grep rp_stamps gpurun_out/stamps_join2.log | head -3
CYLON_RP_STAMPS=1 timeout -k 10 300 python tools/bench_suite.py --configs 5 --reps 1 --scale 0.125 > gpurun_out/stamps_sort2.log 2>&1 || exit 1
grep rp_stamps gpurun_out/stamps_sort2.log | head -3
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_ldsbar.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_ldsbar.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms_max_over_ranks'])"
timeout -k 10 400 python tools/bench_suite.py --configs 4,5,6 --reps 3 > gpurun_out/suite_ldsbar.log 2>&1 || exit 1
grep '^{' gpurun_out/suite_ldsbar.log | cut -c1-150
