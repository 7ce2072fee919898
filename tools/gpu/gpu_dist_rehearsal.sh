# Rehearse tools/bench_dist.py (2 ranks sharing the box's GPU over gloo) + 1-GPU timings.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in groupby sort union; do
  timeout -k 10 200 python tools/bench_dist.py --config $c > gpurun_out/dist_${c}_1.log 2>&1 || { tail -20 gpurun_out/dist_${c}_1.log; exit 1; }
  grep '^{' gpurun_out/dist_${c}_1.log
  CYLON_BENCH_BACKEND=gloo-gpu timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
    tools/bench_dist.py --config $c --rows 40000000 > gpurun_out/dist_${c}_2.log 2>&1 || { tail -20 gpurun_out/dist_${c}_2.log; exit 1; }
  grep '^{' gpurun_out/dist_${c}_2.log
done
