#!/bin/bash
# rd4t: gemm_nt — the next tile's k-tile-1 A DMA issued before the epilogue's stores, which then drain
# under two k-tiles (this tree) vs committed (ab/): tests, GEMM / conv tables, ViT + ResNet interleaved
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_nt 300 0 $T tests/test_gemm_nt_gpu.py tests/test_conv_gpu.py tests/test_linear_gpu.py -m gpu
step gemm_new 300 0 python -u scripts/bench_gemm_nt.py
step gemm_old 300 0 python -u ab/scripts/bench_gemm_nt.py
step conv_new 300 0 python -u scripts/bench_conv_nt.py
step conv_old 300 0 python -u ab/scripts/bench_conv_nt.py
step vit_new_1 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_old_1 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
step r50_new_1 300 0 python -u bench.py --steps 20 --warmup 10
step r50_old_1 300 0 python -u ab/bench.py --steps 20 --warmup 10
step vit_new_2 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step vit_old_2 300 0 python -u ab/bench.py --model vit_b16 --steps 10 --warmup 5
step r50_new_2 300 0 python -u bench.py --steps 20 --warmup 10
step r50_old_2 300 0 python -u ab/bench.py --steps 20 --warmup 10
echo done
