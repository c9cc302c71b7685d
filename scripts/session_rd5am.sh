#!/bin/bash
# round 5: conv3x3n with software-pipelined k-steps (C3N_SWP) vs without, interleaved on one box
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step pytest_c3n 300 0 python -u -m pytest tests/test_conv3x3n_gpu.py -x -q --timeout 120 --timeout-method thread
T="python scripts/diag/time_c3n.py"
for r in 1 2 3; do
  step c3n_swp1_$r 120 0 $T
  step c3n_swp0_$r 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_c3n_swp0.so $T
done
echo done
