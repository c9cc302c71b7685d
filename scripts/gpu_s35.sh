#!/bin/bash
# session 35: BN finalize kernels (64 channels x 4 shard groups, all loads in flight)
source "$(dirname "$0")/gpu_lib.sh"
step pytest_bn 400 0 python -u -m pytest tests/test_batchnorm.py tests/test_fused_block_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_bn_ops 300 0 python scripts/bench_bn_ops.py
step bench_default 400 0 python bench.py
cd /tmp && step prof35 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof35" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
