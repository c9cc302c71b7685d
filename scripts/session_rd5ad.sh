#!/bin/bash
# round 5: ViT-B/16 plain Linears on hipBLASLt (default) vs gemm_nt (FLUXMPI_GEMM_NT=all), with and
# without the emulated RCCL CU footprint (--force-comm at N = 1)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --model vit_b16 --steps 20 --warmup 10 --force-comm"
step v_blas 300 0 $B
step v_nt 300 0 env FLUXMPI_GEMM_NT=all $B
step v_blas_emu 300 0 $B --emulate-comm 64:150:512:32
step v_nt_emu 300 0 env FLUXMPI_GEMM_NT=all $B --emulate-comm 64:150:512:32
step v_blas_emu32 300 0 $B --emulate-comm 32:300:256
step v_nt_emu32 300 0 env FLUXMPI_GEMM_NT=all $B --emulate-comm 32:300:256
step v_blas_b 300 0 $B
step v_nt_b 300 0 env FLUXMPI_GEMM_NT=all $B
echo done
