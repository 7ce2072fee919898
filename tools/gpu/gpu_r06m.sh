# round 6: balanced wave buckets in the radix quantile kernel; merged host reads in the radix join
# (ranking guard + counts, partition flags + skew masks); bounded chunks without the skew sample
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06m}
mkdir -p $O
. tools/gpu/lib.sh
step newtests 900 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "quantile or median or retain or memory_bounded or skew or order or split"
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
step bench 300 python bench.py --steps 20 --warmup 5
step bounded6 900 python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 3 --warmup 3 --retain 0
tail -3 $O/newtests.out
cat $O/quantile.out | cut -c1-300
grep -h '^{' $O/bench.out | cut -c1-600
grep -h summary $O/bounded6.out | cut -c1-400
