#!/bin/bash
# session 21: implicit-GEMM 3x3 conv numerics + speed vs MIOpen
source "$(dirname "$0")/gpu_lib.sh"
step pytest_conv 300 0 python -u -m pytest tests/test_conv_gpu.py -x -v --timeout 120 --timeout-method thread
step bench_conv 300 0 python scripts/bench_conv3x3.py
echo done
