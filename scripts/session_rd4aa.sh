#!/bin/bash
# rd4aa: ViT [CLS] + position embedding in one elementwise pass (no concatenated copy) vs committed (ab/)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_vit 300 0 $T tests/test_vit_gpu.py tests/test_vit_model_gpu.py -m gpu
step vit_new_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_old_1 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
step vit_new_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_old_2 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
step vit_new_3 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_old_3 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
echo done
