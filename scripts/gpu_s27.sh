#!/bin/bash
# session 27: autotuned weight gradients (MIOpen vs our split-K kernel) in the ResNet path
source "$(dirname "$0")/gpu_lib.sh"
step pytest_k 400 0 python -u -m pytest tests/test_conv_gpu.py tests/test_fused_block_gpu.py -x -q --timeout 120 --timeout-method thread
step bench_auto 400 0 python bench.py
FLUXMPI_WGRAD=miopen step bench_wmiopen 400 0 python bench.py
cd /tmp && step prof27 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof27" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
