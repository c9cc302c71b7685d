#!/bin/bash
# rd4ac: gemm_nt XCD-interleaved tile order (FLUXMPI_GEMM_NT_ORDER=1, default) vs contiguous ranges (0):
# tests, GEMM / conv tables, L2 hit counters, ViT + ResNet interleaved
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_nt 400 0 $T tests/test_gemm_nt_gpu.py tests/test_conv_gpu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py tests/test_gelu.py tests/test_layernorm.py -m gpu
step gemm_o1 300 0 python -u scripts/bench_gemm_nt.py
FLUXMPI_GEMM_NT_ORDER=0 step gemm_o0 300 0 python -u scripts/bench_gemm_nt.py
step conv_o1 300 0 python -u scripts/bench_conv_nt.py
FLUXMPI_GEMM_NT_ORDER=0 step conv_o0 300 0 python -u scripts/bench_conv_nt.py
cd /tmp
step pmc_o1 120 0 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
  TCC_HIT_sum TCC_MISS_sum -d "$OUT/pmc_o1" -o run --output-format csv -- python3 "$ROOT/scripts/pmc_gemm_nt.py"
cd "$ROOT"
step vit_o1_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT_ORDER=0 step vit_o0_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step r50_o1_1 300 0 python -u bench.py --steps 20 --warmup 10
FLUXMPI_GEMM_NT_ORDER=0 step r50_o0_1 300 0 python -u bench.py --steps 20 --warmup 10
step vit_o1_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT_ORDER=0 step vit_o0_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step r50_o1_2 300 0 python -u bench.py --steps 20 --warmup 10
FLUXMPI_GEMM_NT_ORDER=0 step r50_o0_2 300 0 python -u bench.py --steps 20 --warmup 10
echo done
