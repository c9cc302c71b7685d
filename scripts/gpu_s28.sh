#!/bin/bash
# session 28: BN-backward reductions in the LDS-DMA GEMM epilogue (BNStatsLink for bn1/bn2/bn3)
source "$(dirname "$0")/gpu_lib.sh"
step pytest_k 400 0 python -u -m pytest tests/test_conv_gpu.py tests/test_fused_block_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_nolink 400 0 python bench.py
FLUXMPI_BN_LINK=1 step bench_link 400 0 python bench.py
echo done
