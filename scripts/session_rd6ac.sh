#!/bin/bash
# round 6: forward Anderson mixing (beta) and Gram regulariser (lam) vs the MNIST residual floor;
# three interleaved rounds per setting (the lines vary run to run)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --model deq --steps 40 --warmup 10"
for r in 1 2 3; do
  step m_b10_$r 300 0 $B
  step m_b08_$r 300 0 $B --deq-solver beta=0.8
  step m_b06_$r 300 0 $B --deq-solver beta=0.6
  step m_l2_$r 300 0 $B --deq-solver lam=1e-2
done
echo done
