#!/bin/bash
# session 32: vectorised BN coefficient prologues + work-sized elementwise grids
source "$(dirname "$0")/gpu_lib.sh"
step pytest_bn 400 0 python -u -m pytest tests/test_batchnorm.py tests/test_fused_block_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_bn_ops 300 0 python scripts/bench_bn_ops.py
step bench_default 400 0 python bench.py
echo done
