# round 6: packed (h2 | row) verification column of the hashed string group-by; then the whole GPU
# suite and the round's headline / quantile / bounded / string numbers on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06r}
mkdir -p $O
. tools/gpu/lib.sh
step sgbtests 600 python -u -m pytest tests/test_gpu_radix_joins.py -x -q --timeout 300 --timeout-method thread -k "hashed_string or string"
step sgb_var 400 python tools/string_groupby_probe.py 200000000 10000000 3 --var=8,32
step bench 300 python bench.py --steps 20 --warmup 5
step pytest 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
step sjoin_var 400 python tools/string_join_probe.py 200000000 3 --var=8,32
tail -2 $O/sgbtests.out $O/pytest.out
cat $O/sgb_var.out $O/quantile.out $O/sjoin_var.out | cut -c1-300
grep -h '^{' $O/bench.out | cut -c1-400
