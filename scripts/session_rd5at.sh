#!/bin/bash
# round 5: conv3x3n 128-channel kernel with a 4 x 2 wave grid (64 rows x 64 channels per wave: 8
# fragment reads per 16 MFMAs instead of 10) vs 8 x 1: numerics of the variant, per-call A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
V=exp/variants/_C_c3n_wn2.so
step pytest_wn2 300 0 env FLUXMPI_C_VARIANT=$V python -u -m pytest tests/test_conv3x3n_gpu.py -x -q --timeout 120 --timeout-method thread
T="python scripts/diag/time_c3n.py"
for r in 1 2 3; do
  step c3n_wn1_$r 120 0 $T
  step c3n_wn2_$r 120 0 env FLUXMPI_C_VARIANT=$V $T
done
echo done
