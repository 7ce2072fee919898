# round 6: var-length string keys, hashed string group-by, radix QUANTILE, shared-key copies,
# CPU-twin oracles; probes at scale; then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
. tools/gpu/lib.sh
step newtests 900 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "variable_length or hashed_string or string_word_key or string_keys or quantile or to_torch or matches_global or lookback_passes_match_exact"
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
step sjoin_var 400 python tools/string_join_probe.py 200000000 3 --var=8,32
step sgb_var 400 python tools/string_groupby_probe.py 200000000 10000000 3 --var=8,32
step pytest 1500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
tail -3 $O/newtests.out $O/pytest.out
cat $O/quantile.out $O/sjoin_var.out $O/sgb_var.out | cut -c1-600
