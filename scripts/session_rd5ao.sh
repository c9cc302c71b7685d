#!/bin/bash
# round 5: conv3x3n 128-channel tail as 32-output-channel workgroups: numerics, per-call A/B against
# FLUXMPI_CONV3X3N_NOTAIL, ResNet-50 step A/B on the same box
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_c3n 300 0 python -u -m pytest tests/test_conv3x3n_gpu.py tests/test_fused_block_gpu.py -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
  step tail_on_$r 240 0 python scripts/diag/conv3x3n_tail.py
  step tail_off_$r 240 0 env FLUXMPI_CONV3X3N_NOTAIL=1 python scripts/diag/conv3x3n_tail.py
done
B="python bench.py --steps 20 --warmup 10"
step resnet_on 300 0 $B
step resnet_off 300 0 env FLUXMPI_CONV3X3N_NOTAIL=1 $B
step resnet_on2 300 0 $B
step resnet_off2 300 0 env FLUXMPI_CONV3X3N_NOTAIL=1 $B
echo done
