#!/bin/bash
# round 5: price of conv3x3n's statistics epilogue: EPI 3 vs EPI 0, and diagnostic builds without the
# 16-lane DPP sums / without the shard atomics
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
T="python scripts/diag/time_c3n.py"
for r in 1 2; do
  step c3s_default_$r 120 0 env C3N_EPI0=1 $T
  for v in norowsum noatomic; do
    step c3s_${v}_$r 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_c3n_$v.so $T
  done
done
echo done
