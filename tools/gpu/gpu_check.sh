set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --rows 100000000 --steps 3 --warmup 1 > gpurun_out/bench_100m.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_1b.log 2>&1
echo "chain exit $?"
tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log gpurun_out/bench_100m.log gpurun_out/bench_1b.log | tail -20
