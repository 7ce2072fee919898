# round 6: quantile GPU tests with the summed-column tolerance, on the folded-reset kernel; smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06zh}
mkdir -p $O
. tools/gpu/lib.sh
step qtests 600 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_ops.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "quantile or median or groupby"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/qtests.out
cat $O/smoke.out
