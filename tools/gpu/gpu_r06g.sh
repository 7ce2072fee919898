# round 6 (re-entry): current tree on the GPU -- whole GPU suite, headline bench + kernel stats,
# quantile / var-length string join + group-by probes (the r06f numbers were lost with the container)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
. tools/gpu/lib.sh
step bench 240 python bench.py --steps 20 --warmup 5
step pytest 1500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
step sjoin_var 400 python tools/string_join_probe.py 200000000 3 --var=8,32
step sgb_var 400 python tools/string_groupby_probe.py 200000000 10000000 3 --var=8,32
step forced 300 env CYLON_SHUFFLE_SELF_RCCL=1 python bench.py --steps 10 --warmup 3 --force-shuffle
step benchprof 400 rocprofv3 --kernel-trace --stats -d $O/bprof -o b -- python bench.py --steps 3 --warmup 1
tail -3 $O/pytest.out
grep -h '^{' $O/bench.out $O/forced.out | cut -c1-700
cat $O/quantile.out $O/sjoin_var.out $O/sgb_var.out | cut -c1-600
