#!/bin/bash
# session 20: downsample-gradient SideGradLink (no add kernel in downsample blocks)
source "$(dirname "$0")/gpu_lib.sh"
step pytest_fb 300 0 python -u -m pytest tests/test_fused_block_gpu.py tests/test_batchnorm.py -m gpu -x -v --timeout 120 --timeout-method thread
step bench_default 400 0 python bench.py
cd /tmp && step prof20 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof20" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
