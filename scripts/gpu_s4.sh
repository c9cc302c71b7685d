#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
build_ext
step pytest_bn 300 1 python -m pytest tests/test_batchnorm.py -m gpu -q -x
step bench_bn 300 0 python scripts/bench_bn.py
export MIOPEN_USER_DB_PATH="$OUT/miopen_db" MIOPEN_CUSTOM_CACHE_DIR="$OUT/miopen_cache"
mkdir -p "$MIOPEN_USER_DB_PATH" "$MIOPEN_CUSTOM_CACHE_DIR"
step find1 600 0 python bench.py --steps 20 --warmup 10 --miopen-find 1
step find2 400 0 python bench.py --steps 20 --warmup 10 --miopen-find 1
du -sh "$MIOPEN_USER_DB_PATH" "$MIOPEN_CUSTOM_CACHE_DIR" > "$OUT/db_sizes.txt"; ls -la "$MIOPEN_USER_DB_PATH" >> "$OUT/db_sizes.txt"
echo done
