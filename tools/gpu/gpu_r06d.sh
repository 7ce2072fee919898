# round 6: quantile fix / sizing, retain = false + chunk-major pass, var-key join profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
. tools/gpu/lib.sh
step newtests 900 python -u -m pytest tests/test_gpu_radix_joins.py -x -q --timeout 200 --timeout-method thread -k "quantile or retain or memory_bounded or variable_length"
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
step retain_headline 600 python tools/retain_probe.py --rows 1000000000 --payload-cols 3 --steps 3 --warmup 1 --retain 0
step retain_headline_kept 600 python tools/retain_probe.py --rows 1000000000 --payload-cols 3 --steps 3 --warmup 1 --retain 1
step bounded6 900 python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 3 --warmup 1 --retain 0
step sjoin_prof 600 rocprofv3 --kernel-trace --stats -d $O/sjoin_prof -o sjoin -- python tools/string_join_probe.py 200000000 2 --var=8,32
grep -h summary $O/retain_headline.out $O/retain_headline_kept.out $O/bounded6.out | cut -c1-400
cat $O/quantile.out | cut -c1-500
tail -3 $O/newtests.out
