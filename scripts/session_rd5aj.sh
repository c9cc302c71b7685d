#!/bin/bash
# round 5: conv3x3n time partition (diagnostic builds: no filter staging / no k-steps / no halo) and
# the distance-2 filter prefetch variant, interleaved on one box
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
T="python scripts/diag/time_c3n.py"
for r in 1 2; do
  step c3n_default_$r 120 0 $T
  for v in nofilter nocompute nohalo pf2; do
    step c3n_${v}_$r 120 0 env FLUXMPI_C_VARIANT=exp/variants/_C_c3n_$v.so $T
  done
done
echo done
