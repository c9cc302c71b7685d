#!/bin/bash
# round 6: Skip DEQ (FastDEQ's explicit initial-guess convolution, trained towards z*) vs the zero
# initial guess: per-step solver iterations under training, and bench lines
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_deq 300 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deq.py
for m in deq deq_cifar; do
  step sk1_$m 300 0 python scripts/diag_deq_contract.py --model $m --steps 40 --solver skip=1,skip_reg=1
  step sk0_$m 300 0 python scripts/diag_deq_contract.py --model $m --steps 40
done
B="python bench.py --steps 20 --warmup 10"
step b_deq_sk1 300 0 $B --model deq --deq-solver skip=1,skip_reg=1
step b_deq_sk0 300 0 $B --model deq
step b_deqc_sk1 300 0 $B --model deq_cifar --deq-solver skip=1,skip_reg=1
step b_deqc_sk0 300 0 $B --model deq_cifar
echo done
