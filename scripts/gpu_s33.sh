#!/bin/bash
# session 33: steady-state profile after the BN prologue fix; ViT and DEQ benches
source "$(dirname "$0")/gpu_lib.sh"
cd /tmp && step prof33 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof33" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
cd "$ROOT" && step bench_vit 300 0 python bench.py --model vit_b16 --steps 10 --warmup 3
step bench_deq 300 0 python bench.py --model deq --steps 10 --warmup 5
echo done
