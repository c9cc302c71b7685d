#!/bin/bash
# rd3s: persistent double-buffered attention forward (FLUXMPI_ATTN_FWD=persist) — tests, ViT A/B, profile
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_attn 300 1 python -u -m pytest tests/test_attention_gpu.py tests/test_vit_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step vit 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_pers 300 0 env FLUXMPI_ATTN_FWD=persist python bench.py --model vit_b16 --steps 20 --warmup 10
step vitb 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_persb 300 0 env FLUXMPI_ATTN_FWD=persist python bench.py --model vit_b16 --steps 20 --warmup 10
cd /tmp && step prof_vit_pers 300 0 env FLUXMPI_ATTN_FWD=persist rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_pers_rd3s" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5; cd "$ROOT"
echo done
