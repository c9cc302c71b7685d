#!/bin/bash
# rd3zf: attention workgroups per head (FLUXMPI_ATTN_PARTS) re-swept with the pipelined <13> kernels
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_p3 300 1 env FLUXMPI_ATTN_PARTS=3 python -u -m pytest tests/test_attention_gpu.py tests/test_vit_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step vit_p2 300 1 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_p1 300 1 env FLUXMPI_ATTN_PARTS=1 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_p3 300 1 env FLUXMPI_ATTN_PARTS=3 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_p4 300 1 env FLUXMPI_ATTN_PARTS=4 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_p2b 300 1 python bench.py --model vit_b16 --steps 20 --warmup 10
echo done
