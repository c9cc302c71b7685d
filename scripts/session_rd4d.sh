#!/bin/bash
# rd4d: stream-K gemm_nt tests + numbers, the DEQ two-forward fix, ViT (fused / all gemm_nt) and ResNet benches
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_gemm_nt 400 0 $T tests/test_gemm_nt_gpu.py
step bench_gemm_nt 400 0 python -u scripts/bench_gemm_nt.py
step test_deq 400 1 $T tests/test_deq.py -m gpu
step bench_vit 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT=all step bench_vit_all 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step bench_vit_fc 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5 --force-comm
step bench_r50 300 0 python -u bench.py --steps 20 --warmup 10
step bench_r50_fc 300 0 python -u bench.py --steps 20 --warmup 10 --force-comm
step bench_deqc 400 0 python -u bench.py --model deq_cifar --batch 128 --steps 10 --warmup 5
step bench_deqc_func 400 0 python -u bench.py --model deq_cifar --batch 128 --steps 10 --warmup 5 --api functional --force-comm
echo done
