#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_gpu 600 1 python -m pytest tests -m gpu -q -x
step bench_default 500 0 python bench.py
mkdir -p "$OUT/miopen_db" && cp /tmp/fluxmpi_miopen_*/rank0/*.txt "$OUT/miopen_db/" || true
step bench_deq 300 0 python bench.py --model deq --image 28 --steps 10 --warmup 5
cd /tmp && step prof_vit 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vit" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_b16 --steps 5 --warmup 3
cd /tmp && step prof14 400 0 rocprofv3 --kernel-trace --stats -d "$OUT/prof14" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 5
echo done
