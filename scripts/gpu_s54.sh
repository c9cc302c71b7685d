#!/bin/bash
# session 54: kernel stats of the ViT-B/16 and DEQ benches
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
cd /tmp && step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
cd /tmp && step prof_deq 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_deq" -o run --output-format csv -- python3 "$ROOT/bench.py" --model deq --steps 5 --warmup 5
echo done
