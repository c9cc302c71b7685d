#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_gpu 600 1 python -m pytest tests -m gpu -q -x
step bench_gemm 400 0 python scripts/bench_gemm.py
step bench_hybrid 400 0 python bench.py --conv hybrid
step bench_miopen 400 0 python bench.py --conv miopen
step bench_fused 400 0 python bench.py --conv fused
cd /tmp && step prof10 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof10" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5 --conv hybrid
echo done
