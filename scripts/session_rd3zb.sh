#!/bin/bash
# rd3zb: explicitly pipelined attention dK/dV kernel (<13, 1>) vs the unrolled one (<13, 0>)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_attn 300 1 python -u -m pytest tests/test_attention_gpu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step vit 300 1 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_nop 300 1 env FLUXMPI_ATTN_DKV_PIPE=0 python bench.py --model vit_b16 --steps 20 --warmup 10
step vitb 300 1 python bench.py --model vit_b16 --steps 20 --warmup 10
step vit_nopb 300 1 env FLUXMPI_ATTN_DKV_PIPE=0 python bench.py --model vit_b16 --steps 20 --warmup 10
cd /tmp && step prof_vit 300 1 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd3zb" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5; cd "$ROOT"
echo done
