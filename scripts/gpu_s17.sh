#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_gpu 600 1 python -m pytest tests -m gpu -q
step bench_default 500 0 python bench.py
step bench_vit 400 0 python bench.py --model vit_b16 --steps 10 --warmup 3
step gemm_tiles 400 0 python scripts/bench_gemm_tiles.py
cd /tmp && step prof17 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof17" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
cd /tmp && step prof_vit 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 3
echo done
