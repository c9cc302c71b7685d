#!/bin/bash
# rd4ad: plain ViT Linears routed per shape by measurement (FLUXMPI_GEMM_NT=measure, new default) vs
# fused-only (previous default) vs all, ViT-B/16 interleaved; tests
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_lin 400 0 $T tests/test_linear_gpu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py tests/test_gemm_nt_gpu.py tests/test_layernorm.py tests/test_gelu.py -m gpu
step vit_measure_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --dump-choices gpurun_out/vit_choices.jsonl
FLUXMPI_GEMM_NT=fused step vit_fused_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_measure_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT=fused step vit_fused_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT=all step vit_all 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
echo done
