#!/bin/bash
# session 59: DEQ adjoint without GroupNorm parameter reductions — tests + bench x2
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_deq 300 0 python -u -m pytest tests/test_deq.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench_deq 300 0 python bench.py --model deq
step bench_deq2 300 0 python bench.py --model deq --steps 40
echo done
