#!/bin/bash
# round 6: linbwd.hip (a Linear's input + weight gradient in one launch): GPU tests, per-shape
# microbench, ViT-B/16 A/B; conv_c3 pipelined filter gradient; DEQ solver diagnosis; roofline BN rows
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step test_new 400 0 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_linbwd_gpu.py tests/test_conv_c3_gpu.py
step bench_linbwd 300 0 python scripts/bench_linbwd.py
B="python bench.py --steps 20 --warmup 10"
step vit_lb1 300 0 env FLUXMPI_LINBWD=1 $B --model vit_b16
step vit_lb0 300 0 env FLUXMPI_LINBWD=0 $B --model vit_b16
step vit_lb1b 300 0 env FLUXMPI_LINBWD=1 $B --model vit_b16
step vit_lb0b 300 0 env FLUXMPI_LINBWD=0 $B --model vit_b16
step test_vit 400 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vit_model_gpu.py tests/test_linear_gpu.py tests/test_vit_gpu.py
step diag_solver_deq 300 0 python scripts/diag_deq_solver.py --model deq --train 40
step diag_solver_deqc 400 0 python scripts/diag_deq_solver.py --model deq_cifar --train 40
step roofline_bn 300 0 env ROOFLINE_BN_ONLY=1 python scripts/roofline_resnet50.py "$OUT/rd6d_roofline_bn.md"
echo done
