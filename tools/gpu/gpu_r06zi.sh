# round 6 final (after the folded-reset QUANTILE kernel and the test tolerance fix): GPU suite, smoke, headline, quantile probe
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06zi}
mkdir -p $O
. tools/gpu/lib.sh
step pytest 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 20 --warmup 5
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
tail -2 $O/pytest.out
cat $O/smoke.out
grep -h '^{' $O/bench.out | cut -c1-400
cat $O/quantile.out | cut -c1-300
