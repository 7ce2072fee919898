# round 6: where the bounded-memory join (1B x 1B, 6 payload columns, retain=false) and the
# variable-length string join / group-by spend their time (kernel traces)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
. tools/gpu/lib.sh
step bounded6 900 python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 3 --warmup 3 --retain 0
step bprof 900 rocprofv3 --kernel-trace --stats -d $O/bprof -o b -- python tools/retain_probe.py --rows 1000000000 --payload-cols 6 --steps 1 --warmup 2 --retain 0
step sjprof 400 rocprofv3 --kernel-trace --stats -d $O/sjprof -o sj -- python tools/string_join_probe.py 200000000 2 --var=8,32
step sgprof 400 rocprofv3 --kernel-trace --stats -d $O/sgprof -o sg -- python tools/string_groupby_probe.py 200000000 10000000 2 --var=8,32
grep -h summary $O/bounded6.out | cut -c1-400
grep -h '"step"' $O/bounded6.out | cut -c1-250
