# Join partition passes with LDS-atomic (unstable) ranking vs the stable ballot ranking:
# join tests, A/B bench, phase stamps of the unstable pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  -k "radix_join or 100m or packed_validity" > gpurun_out/unstable_tests.log 2>&1 || { tail -30 gpurun_out/unstable_tests.log; exit 1; }
tail -3 gpurun_out/unstable_tests.log
for v in 0 1 0 1; do
  CYLON_RP_STABLE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/unstable_bench_$v.log 2>&1 || exit 1
  echo "stable=$v $(tail -1 gpurun_out/unstable_bench_$v.log)"
done
CYLON_RP_STAMPS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-phases > gpurun_out/stamps_unstable.log 2>&1 || exit 1
grep rp_stamps gpurun_out/stamps_unstable.log | head -8
