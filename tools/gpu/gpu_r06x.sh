# round 6 final: N-rank rehearsal of bench.py on one card (gloo-gpu, 2/4/8 ranks, verify on every rank)
# + the headline PMC set on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06x}
mkdir -p $O
. tools/gpu/lib.sh
for N in 2 4 8; do
  step mr$N 400 env CYLON_BENCH_BACKEND=gloo-gpu python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2951$N bench.py --gpus $N --steps 2 --warmup 1 --rows 40000000
done
for N in 2 4 8; do grep -h '^{' $O/mr$N.out | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print('N=$N', round(r['ms_per_step'],1), 'ms', 'verify', r['verify']['ok'], r['verify'].get('rows'), r['verify'].get('expected_rows'), 'ranks', len(r.get('ranks', [])))"; done
bash tools/gpu/gpu_pmc_headline.sh r06 > $O/pmc.log 2>&1 || true
cat gpurun_out/pmc_r06/summary.txt
