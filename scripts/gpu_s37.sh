#!/bin/bash
# session 37: 256x128 LDS-DMA GEMM tiles (engines 7/8) — correctness + shape sweeps
source "$(dirname "$0")/gpu_lib.sh"
step pytest_conv 400 0 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_conv3x3 400 0 env BENCH_ENGINES=2,5,7,8 python scripts/bench_conv3x3.py
step bench_gemm 400 0 env BENCH_ENGINES=2,5,7,8 python scripts/bench_gemm_tiles.py
echo done
