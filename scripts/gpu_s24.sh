#!/bin/bash
# session 24: conv3x3 per-shape forward choice, glds variant rule without the 128x64 switch
source "$(dirname "$0")/gpu_lib.sh"
step pytest_k 400 0 python -u -m pytest tests/test_conv_gpu.py tests/test_fused_block_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_ours 400 0 python bench.py
step bench_conv 300 0 python scripts/bench_conv3x3.py
step bench_tiles 300 0 python scripts/bench_gemm_tiles.py
cd /tmp && step prof24 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof24" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
