#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_gpu 600 1 python -m pytest tests -m gpu -q -x
step bench_bn 300 0 python scripts/bench_bn.py
step bench_gemm 400 0 python scripts/bench_gemm.py
step bench_hybrid 400 0 python bench.py
step bench_miopen 400 0 python bench.py --conv miopen
cd /tmp && step prof11 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof11" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
