# Multi-rank device paths on one GPU (gloo collectives, tables in HBM) + default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_multirank.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_multirank.log; [ $rc -eq 0 ] || exit $rc
CYLON_BENCH_BACKEND=gloo-gpu timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --steps 2 --warmup 1 --rows 20000000 > gpurun_out/bench_gloo_gpu.log 2>&1 || { tail -30 gpurun_out/bench_gloo_gpu.log; exit 1; }
grep '^{' gpurun_out/bench_gloo_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_default.log
