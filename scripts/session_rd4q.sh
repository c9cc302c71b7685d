#!/bin/bash
# rd4q: gemm_nt write-through epilogue stores (FLUXMPI_GEMM_NT_WT auto = K <= 1024) vs plain (0): GEMM
# table, conv shapes, ViT-B/16 and ResNet-50 same-box interleaved
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_nt 300 0 $T tests/test_gemm_nt_gpu.py -m gpu
step gemm_wt 300 0 python -u scripts/bench_gemm_nt.py
FLUXMPI_GEMM_NT_WT=0 step gemm_plain 300 0 python -u scripts/bench_gemm_nt.py
step conv_wt 300 0 python -u scripts/bench_conv_nt.py
FLUXMPI_GEMM_NT_WT=0 step conv_plain 300 0 python -u scripts/bench_conv_nt.py
step vit_wt_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT_WT=0 step vit_plain_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step r50_wt_1 300 0 python -u bench.py --steps 20 --warmup 10
FLUXMPI_GEMM_NT_WT=0 step r50_plain_1 300 0 python -u bench.py --steps 20 --warmup 10
step vit_wt_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT_WT=0 step vit_plain_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step r50_wt_2 300 0 python -u bench.py --steps 20 --warmup 10
FLUXMPI_GEMM_NT_WT=0 step r50_plain_2 300 0 python -u bench.py --steps 20 --warmup 10
echo done
