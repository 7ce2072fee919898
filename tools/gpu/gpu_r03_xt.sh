#!/bin/bash
# XCD-tile pass schedule (CYLON_RP_XT=1): radix GPU tests with XT on, interleaved headline A/B,
# --verify with XT, pass stamps, kernel trace and a FETCH/WRITE counter pass with XT.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03xt
mkdir -p $O
CYLON_RP_XT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py -x -v --timeout 300 --timeout-method thread -k "join or narrow or guard or sort or groupby or set" > $O/pytest.txt 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/base_$i.json 2> $O/base_$i.err
  CYLON_RP_XT=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/xt_$i.json 2> $O/xt_$i.err
done
CYLON_RP_XT=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verify > $O/xt_verify.json 2> $O/xt_verify.err
CYLON_RP_XT=1 CYLON_RP_STAMPS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-phases > $O/stamps_xt.json 2> $O/stamps_xt.err
CYLON_RP_XT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o join -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof.log 2>&1
cd /tmp && export TMPDIR=/tmp
CYLON_RP_XT=1 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_fetch -o f -- python3 $GRAFT_REPO_ROOT/tools/join_probe.py 1000000000 1 > $GRAFT_REPO_ROOT/$O/pmc_fetch.log 2>&1
CYLON_RP_XT=1 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE TCC_EA0_WRREQ_64B_sum --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_write -o w -- python3 $GRAFT_REPO_ROOT/tools/join_probe.py 1000000000 1 > $GRAFT_REPO_ROOT/$O/pmc_write.log 2>&1
cd $GRAFT_REPO_ROOT && python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write k_rows_pass > $O/pmc_summary.txt
echo done
