#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_gemm 300 1 python -m pytest tests/test_gemm_gpu.py tests/test_batchnorm.py -q
step bench_gemm 400 0 python scripts/bench_gemm.py
step bench_bn 300 0 python scripts/bench_bn.py
step bench 400 0 python bench.py
echo done
