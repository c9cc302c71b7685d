#!/bin/bash
# session 26: weight-gradient kernel (transposed LDS-DMA ring, split-K), numerics + speed vs MIOpen
source "$(dirname "$0")/gpu_lib.sh"
step pytest_conv 300 0 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad"
step bench_conv 300 0 python scripts/bench_conv3x3.py
echo done
