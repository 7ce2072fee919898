# Nullable payloads through the radix join (packed validity): device tests + 200M timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_multirank.py -k "nulls or radix or large or identities" > gpurun_out/pt_null.log 2>&1
rc=$?; tail -1 gpurun_out/pt_null.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/nullable_probe.py > gpurun_out/nullable.log 2>&1 || exit 1
grep nullable gpurun_out/nullable.log
