#!/bin/bash
# session 25: 1x1 forward on our GEMM + BN statistics epilogue (per-shape choice)
source "$(dirname "$0")/gpu_lib.sh"
step pytest_k 400 0 python -u -m pytest tests/test_fused_block_gpu.py tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_ours 400 0 python bench.py
FLUXMPI_CONV1X1=miopen step bench_m1 400 0 python bench.py
cd /tmp && step prof25 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof25" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
