# Column-count block-size selection for k_rows_pass: tests + group-by / sort A/B + default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_kernels.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rpsel.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -1 gpurun_out/pytest_rpsel.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_rpsel.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_rpsel.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms_max_over_ranks'])"
for t in auto 1024; do
  if [ $t = auto ]; then unset CYLON_RP_THREADS; else export CYLON_RP_THREADS=$t; fi
  timeout -k 10 400 python tools/bench_suite.py --configs 4,5 --reps 3 > gpurun_out/suite45_$t.log 2>&1 || exit 1
  echo "threads=$t"; grep '^{' gpurun_out/suite45_$t.log | cut -c1-150
done
