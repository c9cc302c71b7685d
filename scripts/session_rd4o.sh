#!/bin/bash
# rd4o: same-box A/B of SLP vectorisation off in attention / gemm_glds / gemm (this tree) vs on (ab/),
# ViT-B/16 and ResNet-50, interleaved; ViT with every Linear on gemm_nt (FLUXMPI_GEMM_NT=all)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_attn_conv 300 0 $T tests/test_attention_gpu.py tests/test_conv_gpu.py tests/test_gemm_nt_gpu.py -m gpu
step vit_noslp_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_slp_1 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
step r50_noslp_1 300 0 python -u bench.py --steps 20 --warmup 10
step r50_slp_1 300 0 python -u ab/bench.py --steps 20 --warmup 10
step vit_noslp_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_slp_2 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
step r50_noslp_2 300 0 python -u bench.py --steps 20 --warmup 10
step r50_slp_2 300 0 python -u ab/bench.py --steps 20 --warmup 10
FLUXMPI_GEMM_NT=all step vit_all 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step nt_exp 300 0 python -u exp/nt_exp.py
echo done
