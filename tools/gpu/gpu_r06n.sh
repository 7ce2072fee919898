# round 6: self-RCCL exchange overlap at 8 vs 16 hash chunks per destination,
# 500M x 500M forced shuffle at world 1 (own rows through RCCL); overlap per step from the kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${RUN:-r06n}
mkdir -p $O
. tools/gpu/lib.sh
for K in 8 16; do
  step ov$K 400 env CYLON_SHUFFLE_SELF_RCCL=1 CYLON_SHUFFLE_CHUNKS=$K rocprofv3 --kernel-trace -d $O/ov$K -o p -- python bench.py --force-shuffle --rows 500000000 --steps 2 --warmup 1
  python tools/overlap_report.py $O/ov$K/p_results.db rcclGenericKernel 3 1 > $O/ov$K.overlap.txt 2>&1 || true
  rm -rf $O/ov$K
  step t$K 300 env CYLON_SHUFFLE_SELF_RCCL=1 CYLON_SHUFFLE_CHUNKS=$K python bench.py --force-shuffle --rows 500000000 --steps 5 --warmup 2
done
for K in 8 16; do echo "== K=$K"; head -6 $O/ov$K.overlap.txt; grep -h '^{' $O/t$K.out | cut -c1-500; done
