#!/bin/bash
# Counter profile of the radix quantile kernel (k_rg_quantile) on tools/quantile_probe.py 1B / 10M:
# one rocprofv3 --pmc pass per counter group, kernel trace only.
set -euo pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
O=$R/gpurun_out/pmc_quantile
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$name -o $name -- python3 $R/tools/quantile_probe.py 1000000000 10000000 1 > $O/$name.log 2>&1
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU
pass sq2 SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU
python3 $R/tools/pmc_summary.py $O/sq $O/sq2 k_rg_quantile > $O/summary.txt 2>&1
python3 $R/tools/pmc_summary.py $O/sq $O/sq2 k_rg_agg >> $O/summary.txt 2>&1
rm -rf $O/sq $O/sq2
echo pmc done
