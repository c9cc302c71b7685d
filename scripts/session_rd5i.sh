#!/bin/bash
# round 5: bf16 Anderson F history — DEQ GPU tests, same-box A/B (fp32 history vs bf16)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
B="--steps 20 --warmup 10"
step pytest_deq 600 0 python -u -m pytest tests/test_deq.py -m gpu -x -q --timeout 120 --timeout-method thread
step deq_f32 300 0 python scripts/diag/bench_deq_f32hist.py --model deq $B
step deq_bf16 300 0 python bench.py --model deq $B
step cifar_f32 300 0 python scripts/diag/bench_deq_f32hist.py --model deq_cifar --force-comm $B
step cifar_bf16 300 0 python bench.py --model deq_cifar --force-comm $B
step deq_f32_b 300 0 python scripts/diag/bench_deq_f32hist.py --model deq $B
step deq_bf16_b 300 0 python bench.py --model deq $B
echo done
