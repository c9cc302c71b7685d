#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
step diag_graphs 300 0 python -u scripts/diag_deq_graphs.py
step pytest_cell 300 1 python -u -m pytest tests/test_deq.py -m gpu -x -v -k "graphs or fused_cell or fused_adjoint" --timeout 120 \
  --timeout-method thread
bash "$(dirname "$0")/session_ab.sh"
