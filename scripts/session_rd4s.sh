#!/bin/bash
# rd4s: steady-state rocprof kernel traces of the current defaults (ResNet-50, ViT-B/16)
source "$(dirname "$0")/gpu_lib.sh"
rm -f "$OUT/steps.log" "$OUT/bench_results.jsonl"
cd /tmp && step prof_r50 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r50_rd4s" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5; cd "$ROOT"
cd /tmp && step prof_vit 300 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit_rd4s" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5; cd "$ROOT"
echo done
