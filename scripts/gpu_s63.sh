#!/bin/bash
# session 63: DEQ kernel trace at the current tree
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
cd /tmp && step prof_deq 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deq63" -o run --output-format csv -- python3 "$ROOT/bench.py" --model deq --steps 5 --warmup 5
echo done
