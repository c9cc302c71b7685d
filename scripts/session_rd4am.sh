#!/bin/bash
# rd4am: ViT-B/16 kernel traces with every Linear on gemm_nt (FLUXMPI_GEMM_NT=all) vs the default
# (fused-only) on the same box: which plain Linears lose in the model
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
cd /tmp
FLUXMPI_GEMM_NT=all step prof_all 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_all" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
step prof_fused 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_fused" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
cd "$ROOT"
echo done
