#!/bin/bash
# round 6: cached placeholder zero in the linked-GELU LayerNorm backward — ViT tests and a steady trace
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step tests 300 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vit_model_gpu.py tests/test_layernorm.py tests/test_vit_gpu.py
step vit 300 0 python bench.py --model vit_b16 --steps 20 --warmup 10
cd /tmp
step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd6ah" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
cd "$ROOT"
echo done
