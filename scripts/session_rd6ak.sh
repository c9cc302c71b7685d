#!/bin/bash
# round 6: Skip DEQ with the skip convolution on a detached injection (the auxiliary loss stops at
# the skip) vs the preset, DEQ-CIFAR, interleaved rounds
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --model deq_cifar --steps 20 --warmup 10"
for r in 1 2 3 4 5; do
  step k_p_$r 300 0 $B
  step k_d_$r 300 0 $B --deq-solver skip_detach=1
done
echo done
