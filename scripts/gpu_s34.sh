#!/bin/bash
# session 34: masked GradLink (bn3 hands (dy, mask) to conv1's dgrad epilogue, no dres pass)
source "$(dirname "$0")/gpu_lib.sh"
step pytest_k 400 0 python -u -m pytest tests/test_fused_block_gpu.py tests/test_gemm_gpu.py tests/test_conv_gpu.py tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_default 400 0 python bench.py
step bench_default2 400 0 python bench.py
echo done
