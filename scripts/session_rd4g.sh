#!/bin/bash
# rd4g: full GPU suite on the round-4 tree, then ResNet (conv rule) and ViT (gemm_nt modes, force-comm delivery)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
step gpu_suite 1000 1 $T tests -m gpu
step bench_r50 300 0 python -u bench.py --steps 20 --warmup 10
FLUXMPI_GEMM_NT_CONV=0 step bench_r50_noconv 300 0 python -u bench.py --steps 20 --warmup 10
step bench_vit 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT=fused step bench_vit_fused 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step bench_vit_fc 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --force-comm
step bench_vit_fc_emu 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --force-comm --emulate-comm 64:300
step bench_r50_fc 300 0 python -u bench.py --steps 20 --warmup 10 --force-comm
echo done
