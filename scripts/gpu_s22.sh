#!/bin/bash
# session 22: LDS-DMA pipelined GEMM (gemm_glds.hip): numerics, conv3x3 + 1x1 + square speed
source "$(dirname "$0")/gpu_lib.sh"
step pytest_conv 300 0 python -u -m pytest tests/test_conv_gpu.py -x -v --timeout 120 --timeout-method thread
step bench_conv 300 0 python scripts/bench_conv3x3.py
step bench_tiles 300 0 python scripts/bench_gemm_tiles.py
echo done
