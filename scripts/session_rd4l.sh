#!/bin/bash
# rd4l: the committed tree (gemm_nt without SLP vectorisation): GEMM / ViT / conv tests, GEMM numbers, benches
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_vit_ops 500 0 $T tests/test_gemm_nt_gpu.py tests/test_gelu.py tests/test_linear_gpu.py tests/test_layernorm.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py tests/test_kernels_gpu.py -m gpu
step bench_gemm_nt 400 0 python -u scripts/bench_gemm_nt.py
step bench_vit 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step bench_r50 300 0 python -u bench.py --steps 20 --warmup 10
echo done
