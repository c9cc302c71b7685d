#!/bin/bash
# round 5: Anderson X / G histories in bf16 (FLUXMPI_DEQ_HIST=bf16): kernel numerics, DEQ / DEQ-CIFAR A/B
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="python bench.py --steps 20 --warmup 10"
step pytest_deq 600 1 python -u -m pytest tests/test_deq.py -m gpu -x -q --timeout 120 --timeout-method thread
step dc_fp32 300 0 $B --model deq_cifar --force-comm
step dc_bf16 300 0 env FLUXMPI_DEQ_HIST=bf16 $B --model deq_cifar --force-comm
step dc_fp32_b 300 0 $B --model deq_cifar --force-comm
step dc_bf16_b 300 0 env FLUXMPI_DEQ_HIST=bf16 $B --model deq_cifar --force-comm
step d_fp32 300 0 $B --model deq
step d_bf16 300 0 env FLUXMPI_DEQ_HIST=bf16 $B --model deq
echo done
