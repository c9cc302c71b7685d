#!/bin/bash
# rd4ag: EPI 2's phase-0/1 derivative loads a k-tile early (this tree) vs committed (ab/): tests, GEMM
# table (both trees), ViT interleaved
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_nt 400 0 $T tests/test_gemm_nt_gpu.py tests/test_vit_gpu.py tests/test_vit_model_gpu.py tests/test_layernorm.py -m gpu
step gemm_new 300 0 python -u scripts/bench_gemm_nt.py
step gemm_old 300 0 python -u ab/scripts/bench_gemm_nt.py
step vit_new_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_old_1 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
step vit_new_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_old_2 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
echo done
