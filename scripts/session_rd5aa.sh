#!/bin/bash
# round 5: wgrad3x3n with 128 output channels per workgroup for the 28x28x128 layers
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_w3n 300 1 python -u -m pytest tests/test_wgrad3x3n_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_w3n 240 0 python scripts/bench_wgrad3x3n.py
echo done
