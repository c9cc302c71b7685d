#!/bin/bash
# round 5: the 128-channel conv3x3n with 16 waves per workgroup (two per 32-row block, 64 output
# channels each: 4 waves per SIMD instead of 2) vs 8: numerics of the variant, per-call A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
V=exp/variants/_C_c3n_w16.so
step pytest_w16 300 0 env FLUXMPI_C_VARIANT=$V python -u -m pytest tests/test_conv3x3n_gpu.py -x -q --timeout 120 --timeout-method thread
T="python scripts/diag/time_c3n.py"
for r in 1 2 3; do
  step c3n_w8_$r 120 0 $T
  step c3n_w16_$r 120 0 env FLUXMPI_C_VARIANT=$V $T
done
echo done
