#!/bin/bash
# round 6: the non-fused adjoint's convergence flag in the reduce launch — DEQ tests and DEQ-CIFAR lines
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step test_deq 300 0 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deq.py
B="python bench.py --steps 20 --warmup 10"
step deq_cifar 300 0 $B --model deq_cifar
step deq_cifar_comm 300 0 $B --model deq_cifar --force-comm
step deq 300 0 $B --model deq
cd /tmp
step prof_deqc 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deqc_rd6y" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --model deq_cifar --steps 5 --warmup 5
cd "$ROOT"
echo done
