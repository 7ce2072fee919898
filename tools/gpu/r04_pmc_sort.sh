#!/bin/bash
# Counter profiles of the 2B-row sort passes (look-back + counting, look-back, counting-only XT),
# one PMC pass per counter group (kernel trace only), counters checked against `rocprofv3 -L`.
# usage: tools/gpu/r04_pmc_sort.sh <tag>
set -euo pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-base}
O=$R/gpurun_out/r04pmcsort_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
pass() {
  local name=$1; shift
  for c in "$@"; do
    grep -q "\b${c%_sum}\b" $O/counters.txt || { echo "counter $c not listed: skip pass $name" >> $O/skipped.txt; return 0; }
  done
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$name -o $name -- python3 $R/tools/bench_suite.py --configs 5 --reps 1 > $O/$name.log 2>&1
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU
pass fetch FETCH_SIZE
pass write WRITE_SIZE TCC_EA0_WRREQ_64B_sum
pass tcc TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum
for k in "k_rows_pass_lean<cylon::hip::ImageDigit, true, 2, true, 3" "k_rows_pass_lean<cylon::hip::ImageDigit, true, 2, true, 2" "k_rows_pass_lean<cylon::hip::ImageDigit, true, 2, true, 1" k_sort_prehist k_lb_reduce k_lb_plan; do python3 $R/tools/pmc_summary.py $O/sq $O/fetch $O/write $O/tcc "$k"; done > $O/summary.txt 2>&1
echo pmc done
