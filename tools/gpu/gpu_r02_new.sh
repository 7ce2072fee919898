# New device tests of this round (bench-scale identities, lists, persistent indexes, graph, sort).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_list_types.py tests/test_gpu_ops.py tests/test_gpu_multirank.py tests/test_arrow_interop.py -m gpu -k "identities or 1b_rows or 2b_rows or list or persistent or streaming or exact_splitters or zero_copy" > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_new.log; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_new.log | tail -25
exit $rc
