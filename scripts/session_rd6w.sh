#!/bin/bash
# round 6: resident attention forward with a 2 TP-row LDS layout (V then K; 53 KB at T = 197) and
# three workgroups per head (FLUXMPI_ATTN_FWD_PARTS, default 3) vs two / one; ViT-B/16 A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_attn 300 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py
step test_attn_p1 300 0 env FLUXMPI_ATTN_FWD_PARTS=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py -k fwd
for r in 1 2; do
  for p in 1 2 3 4; do
    step ba_p${p}_$r 120 0 env FLUXMPI_ATTN_FWD_PARTS=$p python scripts/bench_attn.py
  done
done
B="python bench.py --model vit_b16 --steps 10 --warmup 5"
step vit_p3 300 0 $B
step vit_p2 300 0 env FLUXMPI_ATTN_FWD_PARTS=2 $B
step vit_p3b 300 0 $B
step vit_p2b 300 0 env FLUXMPI_ATTN_FWD_PARTS=2 $B
echo done
