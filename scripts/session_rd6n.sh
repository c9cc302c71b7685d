#!/bin/bash
# round 6: DEQ solver iterations under training at lower Adam learning rates (the converging presets)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for lr in 1e-4 3e-4 1e-3; do
  step lr_deq_$lr 200 0 python scripts/diag_deq_contract.py --model deq --steps 40 --lr $lr
  step lr_deqc_$lr 300 0 python scripts/diag_deq_contract.py --model deq_cifar --steps 40 --lr $lr
done
echo done
