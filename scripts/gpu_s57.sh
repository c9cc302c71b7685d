#!/bin/bash
# session 57: fused NHWC GroupNorm (+add, +ReLU) for the DEQ cell — numerics, bench, kernel trace
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step pytest_deq 300 0 python -u -m pytest tests/test_deq.py -m gpu -x -v --timeout 120 --timeout-method thread
step bench_deq 300 0 python bench.py --model deq
cd /tmp && step prof_deq 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deq57" -o run --output-format csv -- python3 "$ROOT/bench.py" --model deq --steps 5 --warmup 5
echo done
