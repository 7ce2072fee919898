# Packed-validity passes in sort and shuffle: GPU tests + before/after probe timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_kernels.py tests/test_gpu_ops.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_pack.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_pack.log; tail -3 gpurun_out/pytest_pack.log
[ $rc -eq 0 ] || exit $rc
for op in sort shuffle join; do
  timeout -k 10 300 python -u tools/nullable_probe.py --op=$op >> gpurun_out/nullable_pack.log 2>&1 || exit 1
done
cat gpurun_out/nullable_pack.log
for op in sort shuffle join; do
  CYLON_PACK_VALIDITY=0 timeout -k 10 300 python -u tools/nullable_probe.py --op=$op --only-nullable >> gpurun_out/nullable_unpacked.log 2>&1 || exit 1
done
cat gpurun_out/nullable_unpacked.log
