#!/bin/bash
# rd4an: attention workgroups per head (FLUXMPI_ATTN_PARTS) re-swept on the final tree, ViT-B/16 interleaved
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
for r in 1 2; do
  step vit_p2_$r 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
  FLUXMPI_ATTN_PARTS=1 step vit_p1_$r 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
  FLUXMPI_ATTN_PARTS=3 step vit_p3_$r 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
done
echo done
