#!/bin/bash
# session 52: HIP attention forward + backward — numerics, micro-bench, ViT bench, kernel stats
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_attn 200 0 python -u -m pytest tests/test_attention_gpu.py tests/test_vit_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step battn 120 0 python scripts/bench_attn.py
step bench_vit 300 0 python bench.py --model vit_b16
cd /tmp && step prof52 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof52" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
echo done
