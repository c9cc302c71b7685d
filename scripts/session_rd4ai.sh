#!/bin/bash
# rd4ai: gemm_nt epilogue store policy with the interleaved tile order: plain (0) / write-through (1) /
# non-temporal (2): GEMM tables, then ViT for the best candidates
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
FLUXMPI_GEMM_NT_STORE=2 step test_nt 300 0 $T tests/test_gemm_nt_gpu.py -m gpu
step gemm_s0 300 0 python -u scripts/bench_gemm_nt.py
FLUXMPI_GEMM_NT_STORE=1 step gemm_s1 300 0 python -u scripts/bench_gemm_nt.py
FLUXMPI_GEMM_NT_STORE=2 step gemm_s2 300 0 python -u scripts/bench_gemm_nt.py
step vit_s0_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT_STORE=1 step vit_s1_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT_STORE=2 step vit_s2_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_s0_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT_STORE=1 step vit_s1_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT_STORE=2 step vit_s2_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
echo done
