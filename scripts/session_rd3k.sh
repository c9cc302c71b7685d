#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
step pytest_cell 300 1 python -u -m pytest tests/test_deq.py -m gpu -x -v -k "graphs or fused_cell" --timeout 120 \
  --timeout-method thread
step pytest_deq 400 1 python -u -m pytest tests/test_deq.py -m gpu -q --timeout 120 --timeout-method thread
bash "$(dirname "$0")/session_ab.sh"
