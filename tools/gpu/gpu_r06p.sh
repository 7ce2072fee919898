# round 6: first-pass chunk tests; radix quantile single-group value-only sort
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06p}
mkdir -p $O
. tools/gpu/lib.sh
step newtests 900 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "memory_bounded or retain or quantile or median"
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
tail -3 $O/newtests.out
cat $O/quantile.out | cut -c1-300
