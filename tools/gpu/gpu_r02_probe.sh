# Write-kernel probe rounds A/B + kernel traces of the union (config 6) and sort (config 5).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_ops.py tests/test_gpu_multirank.py tests/test_properties.py -k "partition or shuffle or split or lane or stable or sort or gpu_" > gpurun_out/pr_tests.log 2>&1 || { tail -30 gpurun_out/pr_tests.log; exit 1; }
tail -1 gpurun_out/pr_tests.log
for v in "" "CYLON_RJ_PROBE_ROUNDS=2" "" "CYLON_RJ_PROBE_ROUNDS=2"; do
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/pr_bench.log 2>&1 || exit 1
  echo "[$v] $(tail -1 gpurun_out/pr_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), d["phases_ms_max_over_ranks"])')"
done
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg6 -o u -- python3 $GRAFT_REPO_ROOT/tools/bench_suite.py --configs 6 --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_cfg6.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_cfg6/u_results.db 12 > gpurun_out/prof_cfg6_summary.txt; cat gpurun_out/prof_cfg6_summary.txt
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg5 -o s -- python3 $GRAFT_REPO_ROOT/tools/bench_suite.py --configs 5 --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_cfg5.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_cfg5/s_results.db 12 > gpurun_out/prof_cfg5_summary.txt; cat gpurun_out/prof_cfg5_summary.txt
