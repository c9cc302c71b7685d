#!/bin/bash
# round 6: Skip DEQ auxiliary-loss weight 4 vs the preset's 1 (DEQ-CIFAR), interleaved rounds
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --model deq_cifar --steps 20 --warmup 10"
for r in 1 2 3 4 5; do
  step l_p_$r 300 1 $B
  step l_4_$r 300 1 $B --deq-solver skip_reg=4
done
echo done
