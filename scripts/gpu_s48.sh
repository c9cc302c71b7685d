#!/bin/bash
# session 48: ViT-B/16 baseline + ViT kernel stats
source "$(dirname "$0")/gpu_lib.sh"
step bench_vit 400 0 python bench.py --model vit_b16
cd /tmp && step prof48 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof48" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 5
echo done
