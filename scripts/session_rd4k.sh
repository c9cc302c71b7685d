#!/bin/bash
# rd4k: fc1's forward epilogue stores gelu'(h); fc2's dgrad epilogue multiplies by it (no GELU math
# in the backward): tests, GEMM numbers, ViT fused / all / force-comm, ResNet
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_vit_ops 500 0 $T tests/test_gemm_nt_gpu.py tests/test_gelu.py tests/test_linear_gpu.py tests/test_layernorm.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py -m gpu
step bench_gemm_nt 400 0 python -u scripts/bench_gemm_nt.py
step bench_vit 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT=all step bench_vit_all 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step bench_vit_fc 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --force-comm
step bench_vit_fc_emu 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --force-comm --emulate-comm 64:300
step bench_r50 300 0 python -u bench.py --steps 20 --warmup 10
echo done
