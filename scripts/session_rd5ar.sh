#!/bin/bash
# round 5: BN + ReLU + max-pool forward with the 3x3 window at compile time (all nine loads issued
# before the compares) vs the runtime-window loop: numerics, per-call A/B, ResNet-50 A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_bn 300 0 python -u -m pytest tests/test_batchnorm.py tests/test_stem_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  step pool_kk_$r 120 0 python scripts/diag/time_pool.py
  step pool_gen_$r 120 0 env FLUXMPI_POOL_GENERIC=1 python scripts/diag/time_pool.py
done
B="python bench.py --steps 20 --warmup 10"
step resnet_kk 300 0 $B
step resnet_gen 300 0 env FLUXMPI_POOL_GENERIC=1 $B
step resnet_kk2 300 0 $B
step resnet_gen2 300 0 env FLUXMPI_POOL_GENERIC=1 $B
echo done
