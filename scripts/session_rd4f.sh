#!/bin/bash
# rd4f: tile-granular persistent gemm_nt (no stream-K), conv/statistics epilogues: tests, numbers, ResNet/ViT A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_gemm_nt 400 0 $T tests/test_gemm_nt_gpu.py
step bench_conv_nt 400 0 python -u scripts/bench_conv_nt.py
step bench_gemm_nt 400 0 python -u scripts/bench_gemm_nt.py
step bench_r50 300 0 python -u bench.py --steps 20 --warmup 10
FLUXMPI_GEMM_NT_CONV=0 step bench_r50_noconv 300 0 python -u bench.py --steps 20 --warmup 10
step bench_vit 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT=all step bench_vit_all 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step bench_vit_fc 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --force-comm
echo done
