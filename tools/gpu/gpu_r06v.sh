# round 6 final: whole GPU suite, smoke, headline, string join with the scan-based offsets
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06v}
mkdir -p $O
. tools/gpu/lib.sh
step pytest 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 20 --warmup 5
step sjoin_var 400 python tools/string_join_probe.py 200000000 3 --var=8,32
step bounded6 900 python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 3 --warmup 3 --retain 0
tail -2 $O/pytest.out
cat $O/smoke.out
grep -h '^{' $O/bench.out | cut -c1-400
cat $O/sjoin_var.out | cut -c1-700
grep -h summary $O/bounded6.out
