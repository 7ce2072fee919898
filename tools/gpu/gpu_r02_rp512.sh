# Two 512-thread pass blocks per CU vs one 1024-thread block: tests + join/sort A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_kernels.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rp512.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_rp512.log; tail -3 gpurun_out/pytest_rp512.log
[ $rc -eq 0 ] || exit $rc
for t in 512 1024; do
  CYLON_RP_THREADS=$t timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_rp$t.log 2>&1 || exit 1
  echo "threads=$t"; grep '^{' gpurun_out/bench_rp$t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms_max_over_ranks'])"
  CYLON_RP_THREADS=$t timeout -k 10 300 python tools/bench_suite.py --configs 5 --reps 3 > gpurun_out/suite5_rp$t.log 2>&1 || exit 1
  grep '^{' gpurun_out/suite5_rp$t.log | cut -c1-200
done
