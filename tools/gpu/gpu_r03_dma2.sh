#!/bin/bash
# LDS-DMA: write-kernel build staging (16-byte pieces) and the pass kernel's column-1 DMA during
# ranking (CYLON_RP_DMA).  Join + sort + group-by + set-op GPU tests, then interleaved A/B:
# both off / write-DMA only / both on.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03dma2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py -x -v --timeout 300 --timeout-method thread -k "join or narrow or guard or select or sort or groupby or set" > $O/pytest.txt 2>&1
for i in 1 2; do
  CYLON_RJ_DMA=0 CYLON_RP_DMA=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/off_$i.json 2> $O/off_$i.err
  CYLON_RP_DMA=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/wdma_$i.json 2> $O/wdma_$i.err
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/both_$i.json 2> $O/both_$i.err
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verify > $O/both_verify.json 2> $O/both_verify.err
CYLON_RP_STAMPS=1 CYLON_RP_DMA=0 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-phases > $O/stamps_off.json 2> $O/stamps_off.err
CYLON_RP_STAMPS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-phases > $O/stamps_on.json 2> $O/stamps_on.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o join -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof.log 2>&1
echo done
