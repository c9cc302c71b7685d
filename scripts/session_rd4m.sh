#!/bin/bash
# rd4m: gemm_nt EPI 1 storing gelu'(h) (no SLP vectorisation): where the derivative goes wrong, tests,
# GEMM numbers, ViT bench; ResNet-50 with the BatchNorm-backward reductions in the dgrad epilogues (A/B)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step diag_epi1 120 0 python -u scripts/diag_epi1.py
step test_nt 300 1 $T tests/test_gemm_nt_gpu.py -m gpu
step bench_gemm_nt 400 0 python -u scripts/bench_gemm_nt.py
step bench_vit 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_BN_LINK=1 step bench_r50_bnlink 300 0 python -u bench.py --steps 20 --warmup 10
step bench_r50 300 0 python -u bench.py --steps 20 --warmup 10
echo done
