#!/bin/bash
# round 5: wgrad3x3n with the two-block-deep prefetch: numerics, kernel A/B, ResNet-50
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10"
step pytest_w3n 300 1 python -u -m pytest tests/test_wgrad3x3n_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_w3n 240 0 python scripts/bench_wgrad3x3n.py
step resnet 300 0 $B
echo done
