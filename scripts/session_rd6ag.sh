#!/bin/bash
# round 6: Anderson history restarts (restart = 2) on DEQ-CIFAR (Skip DEQ preset), plain and
# --force-comm, interleaved rounds
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --model deq_cifar --steps 20 --warmup 10"
for r in 1 2 3 4; do
  step c_r0_$r 300 0 $B
  step c_r2_$r 300 0 $B --deq-solver restart=2
  step cc_r0_$r 300 0 $B --force-comm
  step cc_r2_$r 300 0 $B --force-comm --deq-solver restart=2
done
echo done
