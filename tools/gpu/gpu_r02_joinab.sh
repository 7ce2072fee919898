# Headline join: auto block size vs forced 1024 on one box, then a kernel-stats profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_join
for t in auto 1024 auto; do
  if [ $t = auto ]; then unset CYLON_RP_THREADS; else export CYLON_RP_THREADS=$t; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-phases > gpurun_out/bench_ab_$t.log 2>&1 || exit 1
  echo "threads=$t"; grep '^{' gpurun_out/bench_ab_$t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])"
done
unset CYLON_RP_THREADS
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_join -o run -- python bench.py --steps 3 --warmup 1 --no-phases > gpurun_out/prof_join.log 2>&1 || exit 1
find gpurun_out/prof_join -name "*kernel_stats.csv" | head -3
