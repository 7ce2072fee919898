# round 6: column-group chunk passes (bounded memory), wave-bitonic radix quantile; kernel traces of
# the bounded join and the var-length string paths (summaries written on the box, databases dropped)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
. tools/gpu/lib.sh
prof() {  # prof <name> <secs> <cmd...>: kernel trace -> per-kernel summary text, database removed
  local name=$1 secs=$2
  shift 2
  step $name $secs rocprofv3 --kernel-trace --stats -d $O/$name -o p -- "$@"
  python tools/rocpd_summary.py $O/$name/p_results.db --top 25 > $O/$name.summary.txt 2>&1 || true
  rm -rf $O/$name
}
step newtests 900 python -u -m pytest tests/test_gpu_radix_joins.py -x -q --timeout 300 --timeout-method thread -k "quantile or memory_bounded or retain"
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
step bounded6 900 python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 3 --warmup 3 --retain 0
prof bprof 900 python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 1 --warmup 2 --retain 0
prof qprof 400 python tools/quantile_probe.py 1000000000 10000000 1
prof sjprof 400 python tools/string_join_probe.py 200000000 2 --var=8,32
prof sgprof 400 python tools/string_groupby_probe.py 200000000 10000000 2 --var=8,32
tail -3 $O/newtests.out
cat $O/quantile.out | cut -c1-300
grep -h summary $O/bounded6.out | cut -c1-400
