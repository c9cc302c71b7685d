#!/bin/bash
# round 5: the 128-channel conv3x3n tail as 16-output-channel workgroups (8 per tile) vs 32 (4 per
# tile): numerics (the tree's build), per-call A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step pytest_c3n 300 0 python -u -m pytest tests/test_conv3x3n_gpu.py tests/test_fused_block_gpu.py -x -q --timeout 120 --timeout-method thread
T="python scripts/diag/time_c3n.py"
for r in 1 2 3; do
  step c3t_16_$r 120 0 $T
  step c3t_32_$r 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_c3n_tail32.so $T
done
echo done
