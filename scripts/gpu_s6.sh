#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_gemm 300 1 python -m pytest tests/test_gemm_gpu.py -q -x
step bench_gemm 400 0 python scripts/bench_gemm.py
echo done
