#!/bin/bash
# rd4e: gemm_nt 32-bit buffer DMA + conv/statistics epilogues: tests, GEMM + conv numbers, ResNet bench A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_gemm_nt 400 0 $T tests/test_gemm_nt_gpu.py
step bench_conv_nt 400 0 python -u scripts/bench_conv_nt.py
step bench_gemm_nt 400 0 python -u scripts/bench_gemm_nt.py
step bench_r50 300 0 python -u bench.py --steps 20 --warmup 10
FLUXMPI_GEMM_NT_CONV=0 step bench_r50_noconv 300 0 python -u bench.py --steps 20 --warmup 10
step bench_vit 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
echo done
