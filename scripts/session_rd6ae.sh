#!/bin/bash
# round 6: more interleaved rounds of Anderson restart = 2 vs none (MNIST DEQ), the rd6ad spread being large
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --model deq --steps 40 --warmup 10"
for r in 1 2 3 4 5 6; do
  step e_r0_$r 300 0 $B
  step e_r2_$r 300 0 $B --deq-solver restart=2
done
echo done
