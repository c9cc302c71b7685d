#!/bin/bash
# session 36: dual BatchNorm for downsample blocks (bn3 + downsample BN in one kernel pair)
source "$(dirname "$0")/gpu_lib.sh"
step pytest_dual 400 0 python -u -m pytest tests/test_fused_block_gpu.py tests/test_batchnorm.py tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_default 400 0 python bench.py
step bench_nodual 400 0 env FLUXMPI_DUAL_BN=0 python bench.py
cd /tmp && step prof36 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof36" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
