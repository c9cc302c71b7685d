#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
step pytest_dv 500 1 python -u -m pytest tests/test_deq.py tests/test_vit_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread
bash "$(dirname "$0")/session_ab.sh"
