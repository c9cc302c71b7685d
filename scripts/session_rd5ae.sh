#!/bin/bash
# round 5: MALL reuse of dY between a 1x1 convolution's weight and input gradients, chunked by pixels
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log"
step chunk_mall 240 0 python scripts/diag/bench_chunk_mall.py
echo done
