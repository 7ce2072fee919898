# After the ranking changes (first join pass: block atomics; stable passes: wave atomics gated by
# the lane-order self-check): GPU suite, smoke, A/B bench, secondary configs, kernel profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
for v in "" "CYLON_RP_RANK=ballot" "" "CYLON_RP_RANK=ballot"; do
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/rk_bench.log 2>&1 || exit 1
  echo "[$v] $(tail -1 gpurun_out/rk_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), d["phases_ms_max_over_ranks"])')"
done
timeout -k 10 900 python -u tools/bench_suite.py --configs 2,4,5,6 --reps 3 > gpurun_out/bench_suite.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_suite.log | cut -c1-200
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_join1b -o join -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-phases > $GRAFT_REPO_ROOT/gpurun_out/prof_join1b.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py gpurun_out/prof_join1b/join_results.db 14 > gpurun_out/prof_join1b_summary.txt; head -12 gpurun_out/prof_join1b_summary.txt
