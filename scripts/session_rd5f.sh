#!/bin/bash
# round 5: BatchNorm-backward finalize folded into the reduce kernels (last-arriver ticket) —
# BN / fused-block tests, the ResNet bench, then the whole GPU suite
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10"
step pytest_bn 600 0 python -u -m pytest tests/test_batchnorm.py tests/test_fused_block_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread
step resnet 300 0 $B
step resnet_b 300 0 $B
step pytest_gpu 900 1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
echo done
