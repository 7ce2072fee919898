set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python tools/bench_suite.py --configs ${CONFIGS:-1,2,4,5} > gpurun_out/bench_suite.log 2>&1; rc=$?
cat gpurun_out/bench_suite.log | grep -v amdgpu.ids; exit $rc
