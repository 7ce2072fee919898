# round 6: first-pass chunks with the merged overflow read (incl. the skewed cases) + bounded probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06w}
mkdir -p $O
. tools/gpu/lib.sh
step newtests 900 python -u -m pytest tests/test_gpu_radix_joins.py -x -q --timeout 300 --timeout-method thread -k "memory_bounded or retain"
step bounded6 900 python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 3 --warmup 3 --retain 0
tail -3 $O/newtests.out
grep -h summary $O/bounded6.out
