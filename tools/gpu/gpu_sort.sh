set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -k "radix or sort" > gpurun_out/pytest_radix.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_radix.log; tail -15 gpurun_out/pytest_radix.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_suite.py --configs 5 > gpurun_out/bench_suite5.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/bench_suite5.log
