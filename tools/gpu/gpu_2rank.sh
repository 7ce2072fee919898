# Two ranks sharing the box's single GPU: rehearses the RCCL multi-rank path (N=2) of bench.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 3 --warmup 1 --rows ${ROWS:-100000000} > gpurun_out/bench_2rank.log 2>&1
rc=$?; tail -15 gpurun_out/bench_2rank.log; exit $rc
