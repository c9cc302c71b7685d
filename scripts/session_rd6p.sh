#!/bin/bash
# round 6: fused attention backward with the K image's first half staged mid-phase-1 (A/B)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_attn 600 0 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_attention_gpu.py tests/test_vit_model_gpu.py
for r in a b; do
  step attn_mid1_$r 120 0 python scripts/bench_attn.py
  step attn_mid0_$r 120 0 env FLUXMPI_ATTN_FUSED_MID=0 python scripts/bench_attn.py
done
B="python bench.py --steps 20 --warmup 10 --model vit_b16"
step vit_mid1 300 0 $B
step vit_mid0 300 0 env FLUXMPI_ATTN_FUSED_MID=0 $B
step vit_mid1b 300 0 $B
step vit_mid0b 300 0 env FLUXMPI_ATTN_FUSED_MID=0 $B
echo done
