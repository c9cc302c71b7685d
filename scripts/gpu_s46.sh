#!/bin/bash
# session 46: compact stride-2 downsample input gradient (residual epilogue with row remap)
source "$(dirname "$0")/gpu_lib.sh"
step pytest_conv 400 0 python -u -m pytest tests/test_conv_gpu.py tests/test_fused_block_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_a 400 0 python bench.py
cd /tmp && step prof46 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof46" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
