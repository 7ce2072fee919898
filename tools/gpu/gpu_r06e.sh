# round 6: pipelined slot pass (RJ_PIPE) first run + A/B, then the GPU suite with it, quantile
# profile, retain / bounded-memory probes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
. tools/gpu/lib.sh
step pipe_small 120 python bench.py --rows 100000000 --steps 3 --warmup 1
step pipe1 180 python bench.py --steps 20 --warmup 5
step classic 180 env CYLON_RJ_PIPE=0 python bench.py --steps 20 --warmup 5
step pipe2 180 python bench.py --steps 20 --warmup 5
step classic2 180 env CYLON_RJ_PIPE=0 python bench.py --steps 20 --warmup 5
step pytest 1500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step quantile_prof 400 rocprofv3 --kernel-trace --stats -d $O/qprof -o q -- python tools/quantile_probe.py 1000000000 10000000 2
step retain0 600 python tools/retain_probe.py --rows 1000000000 --payload-cols 3 --steps 3 --warmup 1 --retain 0
step retain1 600 python tools/retain_probe.py --rows 1000000000 --payload-cols 3 --steps 3 --warmup 1 --retain 1
step bounded6 900 python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 3 --warmup 1 --retain 0
for f in pipe_small pipe1 classic pipe2 classic2; do grep -h '^{' $O/$f.out | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print('$f', r['ms_per_step'], r['phases_ms_max_over_ranks'], r['verify']['ok'])"; done
tail -2 $O/pytest.out
grep -h summary $O/retain0.out $O/retain1.out $O/bounded6.out | cut -c1-400
