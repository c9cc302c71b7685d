#!/bin/bash
# session 60: fused GELU backward + fc1 bias gradient for ViT — numerics, ViT bench, kernel trace
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_gelu 300 0 python -u -m pytest tests/test_gelu.py tests/test_vit_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_vit 300 0 python bench.py --model vit_b16
cd /tmp && step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit60" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
echo done
