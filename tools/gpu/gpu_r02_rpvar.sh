# k_rows_pass variants (CYLON_RP_VARIANT: 0 = 1024 thr, 1 = 2x512 thr/CU, 2 = 768 thr grouped loads x2,
# 3 = 512 thr grouped loads x3 with 256 VGPRs): tests on the default + join/sort A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 2 3; do
  CYLON_RP_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "radix or sort or join or partition" > gpurun_out/pytest_rpvar$v.log 2>&1
  rc=$?; echo "variant $v pytest exit $rc"; tail -1 gpurun_out/pytest_rpvar$v.log
  [ $rc -eq 0 ] || exit $rc
done
for v in 0 1 2 3; do
  CYLON_RP_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_rpvar$v.log 2>&1 || exit 1
  echo "variant=$v"; grep '^{' gpurun_out/bench_rpvar$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms_max_over_ranks'])"
  CYLON_RP_VARIANT=$v timeout -k 10 300 python tools/bench_suite.py --configs 5 --reps 3 > gpurun_out/suite5_rpvar$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/suite5_rpvar$v.log | cut -c1-160
done
