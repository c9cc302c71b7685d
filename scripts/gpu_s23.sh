#!/bin/bash
# session 23: glds GEMM in the ResNet path (1x1 dgrad on cached W^T, implicit-GEMM 3x3 conv2)
source "$(dirname "$0")/gpu_lib.sh"
step pytest_k 400 0 python -u -m pytest tests/test_conv_gpu.py tests/test_fused_block_gpu.py tests/test_gemm_gpu.py tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_ours 400 0 python bench.py
FLUXMPI_CONV3X3=dgrad step bench_dgrad 400 0 python bench.py
FLUXMPI_CONV3X3=miopen step bench_miopen 400 0 python bench.py
step bench_conv 300 0 python scripts/bench_conv3x3.py
cd /tmp && step prof23 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof23" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
