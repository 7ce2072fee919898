# round 6: radix quantile kernel with one HBM round trip per partition, direct group emits and the
# SUM / COUNT / MEAN / MIN / MAX of the quantile's column fused into it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06k}
mkdir -p $O
. tools/gpu/lib.sh
prof() {
  local name=$1 secs=$2
  shift 2
  step $name $secs rocprofv3 --kernel-trace --stats -d $O/$name -o p -- "$@"
  python tools/rocpd_summary.py $O/$name/p_results.db --top 25 > $O/$name.summary.txt 2>&1 || true
  rm -rf $O/$name
}
step newtests 900 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "quantile or median"
step quantile 400 python tools/quantile_probe.py 1000000000 10000000 3
prof qprof 400 python tools/quantile_probe.py 1000000000 10000000 1
tail -3 $O/newtests.out
cat $O/quantile.out | cut -c1-400
head -8 $O/qprof.summary.txt | cut -c1-60,100-170
