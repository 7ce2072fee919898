# round 6: variable-length string keys (join + group-by) tests and probes, default bench, MALL
# reuse go / no-go, then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
. tools/gpu/lib.sh
step newtests 600 python -u -m pytest tests/test_gpu_radix_joins.py -x -q --timeout 200 --timeout-method thread -k "variable_length or hashed_string or string_word_key or string_keys"
step bench 300 python bench.py --steps 20 --warmup 5
step mallreuse 240 ./tools/mallreuse 16
step sjoin_var 400 python tools/string_join_probe.py 200000000 3 --var=8,32
step sgb_var 400 python tools/string_groupby_probe.py 200000000 10000000 3 --var=8,32
step pytest 1200 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -3 $O/newtests.out $O/pytest.out
grep '^{' $O/bench.out | cut -c1-300
cat $O/mallreuse.out $O/sjoin_var.out $O/sgb_var.out | cut -c1-400
