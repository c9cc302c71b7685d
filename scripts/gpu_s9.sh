#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_new 400 1 python -m pytest tests/test_gemm_gpu.py tests/test_fused_block_gpu.py tests/test_batchnorm.py tests/test_ddp_gpu.py -q
step bench_gemm 400 0 python scripts/bench_gemm.py
step bench_fused 400 0 python bench.py --conv fused
step bench_default 400 0 python bench.py
cd /tmp && step prof9 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof9" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5 --conv fused
echo done
