#!/bin/bash
# DEQ session: GPU tests of the DEQ paths, then the same-box A/B list of session_ab.sh
source "$(dirname "$0")/gpu_lib.sh"
step pytest_deq 400 1 python -u -m pytest tests/test_deq.py tests/test_conv_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread
exec_ab() { bash "$(dirname "$0")/session_ab.sh"; }
exec_ab
