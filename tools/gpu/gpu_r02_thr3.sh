# Same-box check: new default vs forced 1024 threads (configs 5, 6).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" "CYLON_RP_THREADS=1024" "CYLON_RP_THREADS=512"; do
  env $v timeout -k 10 600 python -u tools/bench_suite.py --configs 5,6 --reps 3 > gpurun_out/thr3_suite.log 2>&1 || exit 1
  echo "[$v]"; grep '^{' gpurun_out/thr3_suite.log | python -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print("  ", d["config"][:30], d["n"], [round(x,1) for x in d["all_ms"]])'
done
CYLON_RP_STAMPS=1 timeout -k 10 300 python tools/bench_suite.py --configs 6 --reps 1 --scale 0.2 > gpurun_out/stamps_union.log 2>&1 || exit 1
grep rp_stamps gpurun_out/stamps_union.log | head -6
