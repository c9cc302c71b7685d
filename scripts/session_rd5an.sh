#!/bin/bash
# round 5: conv3x3r (C = 64 with the filter resident in LDS, persistent, register-prefetched halo)
# vs the streamed-filter kernel (FLUXMPI_C3N_STREAM64=1): numerics, per-call A/B, ResNet-50 A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_c3n 300 0 python -u -m pytest tests/test_conv3x3n_gpu.py -x -q --timeout 120 --timeout-method thread
T="python scripts/diag/time_c3n.py"
for r in 1 2; do
  step c3r_res_$r 120 0 $T
  step c3r_str_$r 120 0 env FLUXMPI_C3N_STREAM64=1 $T
done
B="python bench.py --steps 20 --warmup 10"
step resnet_res 300 0 $B
step resnet_str 300 0 env FLUXMPI_C3N_STREAM64=1 $B
step resnet_res2 300 0 $B
step resnet_str2 300 0 env FLUXMPI_C3N_STREAM64=1 $B
echo done
