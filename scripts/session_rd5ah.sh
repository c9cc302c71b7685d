#!/bin/bash
# round 5: conv3x3n round quantization probe
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step c3n_tail 240 0 python scripts/diag/conv3x3n_tail.py
echo done
