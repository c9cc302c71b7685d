#!/bin/bash
# rd4x: gemm_nt 128-wide tiles (plain / statistics epilogues; chosen where 256-wide tiles leave a partial
# last round, or N % 256 != 0) and FLUXMPI_GEMM_NT=auto (those plain ViT Linears on gemm_nt) vs the
# committed tree (ab/): tests, GEMM / conv tables (auto vs TN=256), ViT + ResNet interleaved
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_nt 400 0 $T tests/test_gemm_nt_gpu.py tests/test_conv_gpu.py tests/test_linear_gpu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py tests/test_fused_block_gpu.py -m gpu
step gemm_auto 300 0 python -u scripts/bench_gemm_nt.py
FLUXMPI_GEMM_NT_TN=256 step gemm_256 300 0 python -u scripts/bench_gemm_nt.py
step conv_auto 300 0 python -u scripts/bench_conv_nt.py
step vit_new_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_old_1 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
step r50_new_1 300 0 python -u bench.py --steps 20 --warmup 10
step r50_old_1 300 0 python -u ab/bench.py --steps 20 --warmup 10
step vit_new_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_old_2 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
step r50_new_2 300 0 python -u bench.py --steps 20 --warmup 10
step r50_old_2 300 0 python -u ab/bench.py --steps 20 --warmup 10
echo done
