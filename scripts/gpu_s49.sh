#!/bin/bash
# session 49: stem pad kernel, single-pass avg-pool backward, persistent LayerNorm forward,
# packed-QKV attention: their GPU tests, then both benches + ViT kernel stats
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_new 300 0 python -u -m pytest tests/test_resnet_ops_gpu.py tests/test_vit_gpu.py tests/test_layernorm.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_default 400 0 python bench.py
step bench_vit 400 0 python bench.py --model vit_b16
cd /tmp && step prof49 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof49" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
echo done
