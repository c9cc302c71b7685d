#!/bin/bash
# round 5: persistent conv3x3n (next tile's halo prefetched into registers): numerics, then per-call
# A/B against the previous kernel and two schedule variants, interleaved on one box
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step pytest_c3n 300 0 python -u -m pytest tests/test_conv3x3n_gpu.py -x -q --timeout 120 --timeout-method thread
T="python scripts/diag/time_c3n.py"
for r in 1 2; do
  step c3n_new_$r 120 0 $T
  for v in old htap1 u3; do
    step c3n_${v}_$r 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_c3n_$v.so $T
  done
done
echo done
