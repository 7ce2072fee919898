# Ranking variants of the radix pass: LDS-atomic lane-order probe, tests, A/B benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/lds_atomic_order.bin 4096 > gpurun_out/lds_order.log 2>&1; echo "probe exit $?"; cat gpurun_out/lds_order.log
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_kernels.py -k "radix_join or 100m or packed_validity" > gpurun_out/rank_tests.log 2>&1 || { tail -30 gpurun_out/rank_tests.log; exit 1; }
tail -1 gpurun_out/rank_tests.log
CYLON_RP_RANK=wave timeout -k 10 500 $T tests/test_gpu_kernels.py tests/test_gpu_ops.py -k "sort or radix or 100m or set" > gpurun_out/rank_tests_wave.log 2>&1; echo "wave tests exit $?"; tail -3 gpurun_out/rank_tests_wave.log
for v in "" "CYLON_RP_STABLE=1" "CYLON_RP_RANK=wave" ""; do
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/rank_bench.log 2>&1 || exit 1
  echo "[$v] $(tail -1 gpurun_out/rank_bench.log)"
done
for v in "" "CYLON_RP_RANK=wave"; do
  env $v timeout -k 10 400 python tools/bench_suite.py --configs 4,5 --reps 3 > gpurun_out/rank_suite.log 2>&1 || exit 1
  echo "[$v]"; grep -v "^#" gpurun_out/rank_suite.log | tail -4
done
CYLON_RP_STAMPS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-phases > gpurun_out/stamps_rank.log 2>&1 || exit 1
grep rp_stamps gpurun_out/stamps_rank.log | head -4
CYLON_RP_RANK=wave CYLON_RP_STAMPS=1 timeout -k 10 300 python tools/bench_suite.py --configs 5 --reps 1 --scale 0.125 > gpurun_out/stamps_rank_sort.log 2>&1 || exit 1
grep rp_stamps gpurun_out/stamps_rank_sort.log | head -4
