# round 6: radix quantile: 1024 in-partition buckets instead of 2048 (A/B vs r06zd)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06ze}
mkdir -p $O
. tools/gpu/lib.sh
step newtests 900 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "quantile or median"
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
step qprof 400 rocprofv3 --kernel-trace --stats -d $O/qprof -o p -- python tools/quantile_probe.py 1000000000 10000000 1
python tools/rocpd_summary.py $O/qprof/p_results.db --top 25 > $O/qprof.summary.txt 2>&1 || true
rm -rf $O/qprof
tail -3 $O/newtests.out
cat $O/quantile.out | cut -c1-300
head -12 $O/qprof.summary.txt | cut -c1-60,100-170
