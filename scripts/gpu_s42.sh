#!/bin/bash
# session 42: profile after the wgrad XCD-aware grid
source "$(dirname "$0")/gpu_lib.sh"
step bench_a 400 0 python bench.py
cd /tmp && step prof42 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof42" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
cd "$ROOT" && step bench_b 400 0 python bench.py
echo done
