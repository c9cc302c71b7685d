#!/bin/bash
# round 5: narrow 3x3 kernel, split-K tail, optimiser overlap and DEQ-CIFAR delivery — tests first
# (each step bounded; a crash/abort/timeout ends the session), then the GEMM / conv tables and A/Bs
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10"
step pytest_conv_n 240 0 python -u -m pytest tests/test_conv3x3n_gpu.py -m gpu -x -q --timeout 60 --timeout-method thread
step bench_conv_n 240 0 python scripts/bench_conv3x3n.py
step pytest 900 1 python -u -m pytest tests/test_gemm_nt_gpu.py tests/test_ddp_gpu.py tests/test_vit_model_gpu.py \
  tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step resnet 300 0 $B
step resnet_nosplit 300 0 env FLUXMPI_GEMM_NT_SPLIT=0 $B
step bench_nt 600 0 python scripts/bench_gemm_nt.py
step vit 300 0 $B --model vit_b16
step vit_all 300 0 env FLUXMPI_GEMM_NT=all $B --model vit_b16
step vit_comm 300 0 $B --model vit_b16 --force-comm
step vit_comm_ov 300 0 $B --model vit_b16 --force-comm --overlap-opt 1
step resnet_ov 300 0 $B --overlap-opt 1
step deq_cifar 300 0 $B --model deq_cifar --force-comm
step deq_cifar_tol2 300 0 $B --model deq_cifar --force-comm --deq-solver tol=1e-2,bwd_tol=1e-2
step deq_cifar_tol3 300 0 $B --model deq_cifar --force-comm --deq-solver tol=1e-3,bwd_tol=1e-3
