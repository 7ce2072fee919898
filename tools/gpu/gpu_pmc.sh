# Counter profile of the radix-join kernels (two PMC passes, kernel trace only).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p1 -o p1 -- python3 $R/tools/join_probe.py 200000000 2 > $R/gpurun_out/pmc/p1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p2 -o p2 -- python3 $R/tools/join_probe.py 200000000 2 > $R/gpurun_out/pmc/p2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 -L > $R/gpurun_out/pmc/counters.txt 2>&1
ls -R $R/gpurun_out/pmc | head -30
