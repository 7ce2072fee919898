# round 6: selection-based radix QUANTILE, text-mode var-length string keys: tests + probes + profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
. tools/gpu/lib.sh
step newtests 900 python -u -m pytest tests/test_gpu_radix_joins.py -x -q --timeout 200 --timeout-method thread -k "quantile or variable_length or hashed_string or string_word_key or string_keys or retain or memory_bounded or to_torch"
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
step sjoin_var 400 python tools/string_join_probe.py 200000000 3 --var=8,32
step sjoin_prof 400 rocprofv3 --kernel-trace --stats -d $O/sjprof -o sj -- python tools/string_join_probe.py 200000000 1 --var=8,32
step qprof 400 rocprofv3 --kernel-trace --stats -d $O/qprof -o q -- python tools/quantile_probe.py 1000000000 10000000 1
tail -3 $O/newtests.out
cat $O/quantile.out $O/sjoin_var.out | cut -c1-500
