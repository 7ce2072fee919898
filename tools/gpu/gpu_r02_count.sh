# 512-thread join count kernel (two blocks per CU): join tests, bench, kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_kernels.py tests/test_gpu_multirank.py -k "join or 100m" > gpurun_out/cnt_tests.log 2>&1 || { tail -40 gpurun_out/cnt_tests.log; exit 1; }
tail -1 gpurun_out/cnt_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/cnt_bench.log 2>&1 || exit 1
  echo "$(tail -1 gpurun_out/cnt_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), d["phases_ms_max_over_ranks"])')"
done
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_cnt -o join -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-phases > $GRAFT_REPO_ROOT/gpurun_out/prof_cnt.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_cnt/join_results.db 14 > gpurun_out/prof_cnt_summary.txt; head -8 gpurun_out/prof_cnt_summary.txt
