# round 6: where the variable-length string join spends its time (trace phases + kernel stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06t}
mkdir -p $O
. tools/gpu/lib.sh
step sjoin_var 400 python tools/string_join_probe.py 200000000 3 --var=8,32
step sjprof 400 rocprofv3 --kernel-trace --stats -d $O/sjprof -o p -- python tools/string_join_probe.py 200000000 1 --var=8,32
python tools/rocpd_summary.py $O/sjprof/p_results.db --top 40 > $O/sjprof.summary.txt 2>&1 || true
rm -rf $O/sjprof
cat $O/sjoin_var.out | cut -c1-1500
