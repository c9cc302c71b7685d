#!/bin/bash
# session 18: re-validate the rebuilt tree (fresh container), default bench, profile
source "$(dirname "$0")/gpu_lib.sh"
step pytest_gpu 600 1 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 300 0 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 500 0 python bench.py
step gemm_tiles 400 0 python scripts/bench_gemm_tiles.py
step bench_vit 400 0 python bench.py --model vit_b16 --steps 10 --warmup 3
step bench_deq 400 0 python bench.py --model deq --steps 10 --warmup 3
cd /tmp && step prof18 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof18" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
