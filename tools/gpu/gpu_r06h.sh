# round 6: radix quantile kernel (rows as 16-B pairs, 4-row rank rounds, 2 blocks / CU), fused
# shuffle descriptor (counts + key min/max in one read), bounded memory under expandable segments,
# and the deferred-loading crash traced with faulthandler (last: a host segfault ends the script)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
. tools/gpu/lib.sh
step qtests 600 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "quantile"
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
step qprof 400 rocprofv3 --kernel-trace --stats -d $O/qprof -o q -- python tools/quantile_probe.py 1000000000 10000000 1
step forced 300 python bench.py --steps 10 --warmup 3 --force-shuffle
step rccl_tests 600 python -u -m pytest tests/test_gpu_rccl_forced.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread
step bounded6x 900 env PYTORCH_HIP_ALLOC_CONF=expandable_segments:True python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 3 --warmup 1 --retain 0
step deferred 300 env HIP_ENABLE_DEFERRED_LOADING=0 python -X faulthandler bench.py --steps 3 --warmup 1
tail -3 $O/qtests.out $O/rccl_tests.out
cat $O/quantile.out | cut -c1-400
grep -h '^{' $O/forced.out | cut -c1-800
grep -h summary $O/bounded6x.out | cut -c1-400
tail -30 $O/deferred.err
