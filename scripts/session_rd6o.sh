#!/bin/bash
# round 6: fused attention backward (one kernel: S / dP / dS once, dQ from an LDS dS image) —
# numerics vs fp32, per-call time vs the dq / dkv pair, ViT-B/16 A/B; re-check of the DDP / Linear /
# stem tests after the round-6 pruning
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_attn 600 0 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_attention_gpu.py
step test_rest 600 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ddp_gpu.py tests/test_linbwd_gpu.py tests/test_stem_gpu.py tests/test_linear_gpu.py
step attn_pair 120 0 python scripts/bench_attn.py
step attn_fused 120 0 env FLUXMPI_ATTN_BWD=fused python scripts/bench_attn.py
step attn_pair_b 120 0 python scripts/bench_attn.py
step attn_fused_b 120 0 env FLUXMPI_ATTN_BWD=fused python scripts/bench_attn.py
B="python bench.py --steps 20 --warmup 10 --model vit_b16"
step vit_pair 300 0 $B
step vit_fused 300 0 env FLUXMPI_ATTN_BWD=fused $B
step vit_pair_b 300 0 $B
step vit_fused_b 300 0 env FLUXMPI_ATTN_BWD=fused $B
echo done
