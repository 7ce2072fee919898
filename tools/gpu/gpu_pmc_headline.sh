#!/bin/bash
# Counter profile of the 1B x 1B headline join kernels (partition passes, k_rj_count, k_rj_write):
# one rocprofv3 --pmc pass per counter group (kernel trace only; each group within the per-block
# counter limits), counters checked against `rocprofv3 -L`.  usage: tools/gpu/gpu_pmc_headline.sh <tag>
set -euo pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-head}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
pass() {
  local name=$1; shift
  for c in "$@"; do
    grep -q "\b${c%_sum}\b" $O/counters.txt || { echo "counter $c not listed: skip pass $name" >> $O/skipped.txt; return 0; }
  done
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$name -o $name -- python3 $R/tools/join_probe.py 1000000000 1 > $O/$name.log 2>&1
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU
pass sq2 SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU
pass fetch FETCH_SIZE
pass write WRITE_SIZE TCC_EA0_WRREQ_64B_sum
pass tcc TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum
for k in "k_rows_pass<cylon::hip::PartDigitN" k_rj_count k_rj_write k_sl_segments; do
  python3 $R/tools/pmc_summary.py $O/sq $O/sq2 $O/fetch $O/write $O/tcc "$k"
done > $O/summary.txt 2>&1
# the raw per-pass CSVs are large: only the summary and the logs travel back
rm -rf $O/sq $O/sq2 $O/fetch $O/write $O/tcc
echo pmc done
