#!/bin/bash
# LDS-DMA build staging in the join write kernel: join GPU tests, interleaved headline A/B
# (CYLON_RJ_DMA=0 = register staging), phase stamps of both, and a kernel trace of the default.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03dma
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py -x -v --timeout 300 --timeout-method thread -k "join or narrow or guard or select" > $O/pytest.txt 2>&1
for i in 1 2; do
  CYLON_RJ_DMA=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/reg_$i.json 2> $O/reg_$i.err
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/dma_$i.json 2> $O/dma_$i.err
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verify > $O/dma_verify.json 2> $O/dma_verify.err
CYLON_RJ_STAMPS=1 CYLON_RJ_DMA=0 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-phases > $O/stamps_reg.json 2> $O/stamps_reg.err
CYLON_RJ_STAMPS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-phases > $O/stamps_dma.json 2> $O/stamps_dma.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o join -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof.log 2>&1
echo done
