#!/bin/bash
# session 41: wgrad grid 1-D with XCD-aware (split, tile) order
source "$(dirname "$0")/gpu_lib.sh"
step pytest_conv 400 0 python -u -m pytest tests/test_conv_gpu.py tests/test_fused_block_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_conv3x3 400 0 env BENCH_ENGINES=2 python scripts/bench_conv3x3.py
step bench_default 400 0 python bench.py
echo done
