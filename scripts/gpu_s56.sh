#!/bin/bash
# session 56: DEQ activation layout A/B (channels_last vs NCHW-contiguous) + NCHW kernel trace
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
step bench_deq_cl 300 0 python bench.py --model deq --memory-format channels_last
step bench_deq_nchw 300 0 python bench.py --model deq --memory-format contiguous
cd /tmp && step prof_deq 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deq56" -o run --output-format csv -- python3 "$ROOT/bench.py" --model deq --memory-format contiguous --steps 5 --warmup 5
echo done
