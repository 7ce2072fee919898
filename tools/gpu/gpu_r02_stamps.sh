# Phase stamps of k_rows_pass (debug build path, CYLON_RP_STAMPS=1): join passes (4 columns,
# 1024 threads) and the key-only sort passes (1 column, 512 threads), plus 1024-thread sort.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
CYLON_RP_STAMPS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-phases > gpurun_out/stamps_join.log 2>&1 || exit 1
grep rp_stamps gpurun_out/stamps_join.log | head -8
CYLON_RP_STAMPS=1 timeout -k 10 300 python tools/bench_suite.py --configs 5 --reps 1 --scale 0.125 > gpurun_out/stamps_sort.log 2>&1 || exit 1
grep rp_stamps gpurun_out/stamps_sort.log | head -8
CYLON_RP_THREADS=1024 CYLON_RP_STAMPS=1 timeout -k 10 300 python tools/bench_suite.py --configs 5 --reps 1 --scale 0.125 > gpurun_out/stamps_sort1024.log 2>&1 || exit 1
grep rp_stamps gpurun_out/stamps_sort1024.log | head -8
