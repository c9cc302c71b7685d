#!/bin/bash
# session 45: full GPU test suite + bench with the widened weight-gradient autotune
source "$(dirname "$0")/gpu_lib.sh"
step pytest_all 900 0 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_default 400 0 python bench.py
echo done
