# round 6: non-temporal payload loads in the join slot passes, interleaved same-box A/B on the headline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06s}
mkdir -p $O
. tools/gpu/lib.sh
step base1 240 python bench.py --steps 20 --warmup 5
step nt1 240 env CYLON_RJ_NT_LOADS=1 python bench.py --steps 20 --warmup 5
step base2 240 python bench.py --steps 20 --warmup 5
step nt2 240 env CYLON_RJ_NT_LOADS=1 python bench.py --steps 20 --warmup 5
for f in base1 nt1 base2 nt2; do grep -h '^{' $O/$f.out | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print('$f', round(r['ms_per_step'],2), r['phases_ms_max_over_ranks'], r['verify']['ok'])"; done
