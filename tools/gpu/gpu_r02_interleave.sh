# Interleaved (row-major) payload records through the join's partition passes: tests, A/B, stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_kernels.py tests/test_gpu_multirank.py -k "join or 100m" > gpurun_out/il_tests.log 2>&1 || { tail -40 gpurun_out/il_tests.log; exit 1; }
tail -1 gpurun_out/il_tests.log
for v in "" "CYLON_RADIX_INTERLEAVE=0" "CYLON_RP_RANK=wave" "" "CYLON_RADIX_INTERLEAVE=0"; do
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/il_bench.log 2>&1 || exit 1
  echo "[$v] $(tail -1 gpurun_out/il_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), d["phases_ms_max_over_ranks"])')"
done
CYLON_RP_STAMPS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-phases > gpurun_out/stamps_il.log 2>&1 || exit 1
grep rp_stamps gpurun_out/stamps_il.log | head -4
