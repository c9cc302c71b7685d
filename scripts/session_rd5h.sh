#!/bin/bash
# round 5: split-K tail share sweep per ViT GEMM shape, and ViT with every Linear on gemm_nt at
# the larger shares
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10 --model vit_b16"
step bench_nt 600 0 python scripts/bench_gemm_nt.py
step vit 300 0 $B
step vit_all_s16 300 0 env FLUXMPI_GEMM_NT=all FLUXMPI_GEMM_NT_SPLIT=16 $B
step vit_all_s24 300 0 env FLUXMPI_GEMM_NT=all FLUXMPI_GEMM_NT_SPLIT=24 $B
step vit_s24 300 0 env FLUXMPI_GEMM_NT_SPLIT=24 $B
step vit_b 300 0 $B
echo done
