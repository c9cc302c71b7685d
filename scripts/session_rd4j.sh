#!/bin/bash
# rd4j: fp32-param / bf16-grad fused Adam (functional DEQ bench), conv shapes re-measured with the
# 16-B epilogue, ViT default fused, DEQ lines, steady-state rocprof profiles
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step test_kernels 400 0 $T tests/test_kernels_gpu.py tests/test_gemm_nt_gpu.py
step bench_conv_nt 400 0 python -u scripts/bench_conv_nt.py
step bench_deqc_func 400 0 python -u bench.py --model deq_cifar --batch 128 --steps 10 --warmup 5 --api functional --force-comm
step bench_deqc 400 0 python -u bench.py --model deq_cifar --batch 128 --steps 10 --warmup 5 --force-comm
step bench_deq 400 0 python -u bench.py --model deq --steps 10 --warmup 5
step bench_vit 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
FLUXMPI_GEMM_NT=dgrad step bench_vit_dgrad 300 0 python -u bench.py --model vit_b16 --steps 10 --warmup 5
step bench_r50 300 0 python -u bench.py --steps 20 --warmup 10
cd /tmp && step prof_r50 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50_rd4j" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5; cd "$ROOT"
cd /tmp && step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd4j" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5; cd "$ROOT"
echo done
