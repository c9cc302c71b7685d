#!/bin/bash
# session 29: full GPU suite after the LDS-DMA epilogue/prologue variants; default bench
source "$(dirname "$0")/gpu_lib.sh"
step pytest_gpu 600 0 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_default 400 0 python bench.py
echo done
