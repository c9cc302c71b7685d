#!/bin/bash
# round 6: stride-2 3x3 input gradient on the parity-class implicit GEMM (tests, ResNet-50 A/B,
# steady trace), DEQ-CIFAR line
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step test_s2 400 0 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_s2_dgrad_gpu.py tests/test_conv_gpu.py tests/test_resnet_ops_gpu.py
B="python bench.py --steps 20 --warmup 10"
step r50_s2on 300 0 env FLUXMPI_S2_DGRAD=1 $B
step r50_s2off 300 0 env FLUXMPI_S2_DGRAD=0 $B
step r50_s2onb 300 0 env FLUXMPI_S2_DGRAD=1 $B
step r50_s2offb 300 0 env FLUXMPI_S2_DGRAD=0 $B
step deq_cifar 300 0 $B --model deq_cifar --force-comm
cd /tmp
step prof_r50 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50_rd6e" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 5
cd "$ROOT"

step test_lb 300 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linbwd_gpu.py
step bench_linbwd 300 0 python scripts/bench_linbwd.py
step vit 300 0 $B --model vit_b16
step vit_lb0 300 0 env FLUXMPI_LINBWD=0 $B --model vit_b16
step diag_solver_deq 300 0 python scripts/diag_deq_solver.py --model deq --train 40
step diag_solver_deqc 400 0 python scripts/diag_deq_solver.py --model deq_cifar --train 40
step roofline_bn 300 0 env ROOFLINE_BN_ONLY=1 python scripts/roofline_resnet50.py "$OUT/rd6e_roofline_bn.md"
echo done2
