# round 6, first call: GPU suite on the restored tree, default bench, MALL reuse go / no-go
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
. tools/gpu/lib.sh
step mallreuse 240 ./tools/mallreuse 16
step bench 300 python bench.py --steps 20 --warmup 5
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tail -3 $O/pytest.out
grep '^{' $O/bench.out | cut -c1-400
cat $O/mallreuse.out
