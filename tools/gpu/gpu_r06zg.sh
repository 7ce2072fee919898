# round 6: same-box A/B of the radix quantile kernel: HEAD (ab/old) vs the per-partition reset folded
# into the previous partition's trailing barrier (ab/new), ABAB; the quantile GPU tests on the new one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06zg}
mkdir -p $O
. tools/gpu/lib.sh
cp ab/new/libcylon_amd.so cylon_amd/libcylon_amd.so
step newtests 600 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "quantile or median"
cp ab/old/libcylon_amd.so cylon_amd/libcylon_amd.so
step qold1 400 python tools/quantile_probe.py 1000000000 10000000 3
cp ab/new/libcylon_amd.so cylon_amd/libcylon_amd.so
step qnew1 400 python tools/quantile_probe.py 1000000000 10000000 3
cp ab/old/libcylon_amd.so cylon_amd/libcylon_amd.so
step qold2 400 python tools/quantile_probe.py 1000000000 10000000 3
cp ab/new/libcylon_amd.so cylon_amd/libcylon_amd.so
step qnew2 400 python tools/quantile_probe.py 1000000000 10000000 3
tail -1 $O/newtests.out
for f in qold1 qnew1 qold2 qnew2; do echo "== $f"; cut -c1-120 $O/$f.out; done
