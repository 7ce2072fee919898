# Kernel-trace profiles of the secondary configs (5: table sort, 6: union, 4: group-by)
# plus a fresh bench-suite run.  One rocprofv3 run per config so each summary is
# attributable to one workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in 5 6 4; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg$cfg -o cfg \
     -- python3 $GRAFT_REPO_ROOT/tools/bench_suite.py --configs $cfg --reps 1 \
     > $GRAFT_REPO_ROOT/gpurun_out/prof_cfg$cfg.log 2>&1) || exit 1
  python tools/prof_summary.py gpurun_out/prof_cfg$cfg/cfg_results.db 25 > gpurun_out/prof_cfg${cfg}_summary.txt || exit 1
  head -8 gpurun_out/prof_cfg${cfg}_summary.txt
done
timeout -k 10 900 python tools/bench_suite.py --configs 1,2,4,5,6,7 > gpurun_out/bench_suite.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/bench_suite.log
