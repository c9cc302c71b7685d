#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_gpu 400 1 python -m pytest tests -m gpu -q
step bench_default 400 0 python bench.py
step bench_graph 400 0 python bench.py --graph
cd /tmp && step prof5 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof5" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 3
echo done
