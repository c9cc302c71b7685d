#!/bin/bash
# round 6: Anderson history restarts on a stall (restart = 2 / 3 period tests) vs none on the MNIST
# DEQ's trained-cell solves; three interleaved rounds (the lines vary run to run)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_deq 300 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deq.py
B="python bench.py --model deq --steps 40 --warmup 10"
for r in 1 2 3; do
  step m_r0_$r 300 0 $B
  step m_r2_$r 300 0 $B --deq-solver restart=2
  step m_r3_$r 300 0 $B --deq-solver restart=3
done
C="python bench.py --model deq_cifar --steps 20 --warmup 10"
step c_r0 300 0 $C
step c_r2 300 0 $C --deq-solver restart=2
echo done
