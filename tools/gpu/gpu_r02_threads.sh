# Pass block size A/B for narrow passes now that ranking is cheap (sort, group-by, union).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" "CYLON_RP_THREADS=1024" "" "CYLON_RP_THREADS=1024"; do
  env $v timeout -k 10 600 python -u tools/bench_suite.py --configs 4,5,6 --reps 3 > gpurun_out/thr_suite.log 2>&1 || exit 1
  echo "[$v]"; grep '^{' gpurun_out/thr_suite.log | python -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print("  ", d["config"][:40], d["n"], round(d["ms"],2))'
done
